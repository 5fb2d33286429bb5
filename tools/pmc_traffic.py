"""Per-launch HBM traffic of the libsmmd_hip kernels from rocprofv3 PMC passes.

    python tools/pmc_traffic.py <fetch_counter_collection.csv> <write_counter_collection.csv> [out.json]

FETCH_SIZE and WRITE_SIZE are in KB.  On gfx950 FETCH_SIZE reports exactly
half of the bytes of a wide coalesced streaming read (MI355X_MICROARCH.md,
HBM section), so read bytes = 2 * FETCH_SIZE * 1024; WRITE_SIZE is exact for
16-B-per-lane streaming stores.  Kernels are grouped per library entry point
(the launches one call issues) and averaged per call.
"""
import csv
import json
import os
import sys
from collections import defaultdict

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from stamp import library_stamp  # noqa: E402

GROUPS = {
    'smmd_sn_power_iter': ('sn_p1_kernel', 'sn_p2_kernel', 'sn_r2_kernel', 'sn_p3_kernel'),
    'smmd_sn_weight_bwd': ('sn_bwd_a_kernel', 'sn_bwd_b_kernel'),
    'smmd_sn_grad_stats': ('sn_gstat_a_kernel', 'sn_gstat_r_kernel'),
    'smmd_smmd_loss_fwd': ('smmd_loss_kernel',),
    # the fused loss's backward runs scaled_loss_bwd_kernel too: in a run of
    # the fused path this entry is that backward
    'smmd_smmd_loss_bwd': ('scaled_loss_bwd_kernel',),
    'smmd_bn_relu_fwd': ('bn_stats_kernel', 'bn_apply_kernel'),
    'smmd_bn_relu_bwd': ('bn_bwd_stats_kernel', 'bn_bwd_apply_kernel'),
    'smmd_adam_flat': ('opt_sqsum@opt_adam_kernel', 'opt_adam_kernel'),
    'smmd_adam_flat_sn': ('opt_sqsum@opt_adam_sn_kernel', 'opt_adam_sn_kernel'),
    'smmd_clip_by_norm_flat': ('opt_sqsum@opt_clip_kernel', 'opt_clip_kernel'),
    'smmd_mmd2_fwd': ('mmd2_fused_kernel', 'mmd2_tile_kernel'),
    'smmd_scaled_loss_fwd': ('sqnorm_partial_kernel',),
    'smmd_scaled_loss_bwd': ('scaled_loss_bwd_kernel',),
    'smmd_fold_pool_weights': ('fold_fwd_kernel', 'fold_adj_kernel'),
    'smmd_channel_sum': ('chan_sum_partial_kernel', 'chan_sum_final_kernel'),
    'smmd_conv3x3_thin': ('thin_in_kernel', 'thin_out_kernel'),
    'smmd_conv3x3_thin_wgrad': ('thin_wgrad_mfma_kernel', 'thin_wgrad_kernel',
                                'thin_wgrad_final_kernel'),
    'smmd_wino3x3_conv': ('wino_conv_kernel', 'wino_conv8_kernel', 'wino_reduce_kernel'),
    'smmd_wino3x3_filter': ('wino_filter_kernel',),
    'smmd_wino3x3_wgrad': ('wino_wgrad_kernel', 'wino_wgrad2_kernel', 'wino_wgrad_group_kernel',
                           'wino_wgrad_final_kernel', 'wino_wgrad_sum_kernel'),
    'smmd_wino4x4s2_conv': ('s2_conv_kernel',),
    'smmd_wino4x4s2t_conv': ('s2t_conv_kernel',),
    'smmd_wino4x4s2_filter': ('s2_filter_kernel', 's2t_filter_kernel'),
    'smmd_wino4x4s2_wgrad': ('s2_wgrad_kernel', 's2w_sum_kernel', 's2w_group_kernel'),
    'smmd_sn_clip_g': ('sn_clip_g_kernel',),
}
# entry points whose calls each run ONE of their kernels (fold or adjoint;
# thin_in or thin_out):
# calls = the sum of the kernels' launches, not the most frequent one's
SUM_CALLS = ('smmd_fold_pool_weights', 'smmd_conv3x3_thin')


def per_kernel(path):
    """kernel name -> (sum of the counter over its launches, launches); the
    norm pass (opt_sqsum) is attributed, launch by launch, to the update kernel
    dispatched after it (the plain generator update and the SN-fused critic
    update both start with one), under the pseudo-names 'opt_sqsum@<update>'."""
    rows = [r for r in csv.DictReader(open(path)) if 'smmd::' in r['Kernel_Name']]
    rows.sort(key=lambda r: int(r['Dispatch_Id']))
    acc = defaultdict(list)
    for i, r in enumerate(rows):
        name = r['Kernel_Name']
        if 'opt_sqsum_kernel' in name:
            nxt = next((q['Kernel_Name'] for q in rows[i + 1:]
                        if 'opt_adam' in q['Kernel_Name'] or 'opt_clip' in q['Kernel_Name']), '')
            tag = ('opt_adam_sn_kernel' if 'opt_adam_sn' in nxt else
                   'opt_adam_kernel' if 'opt_adam' in nxt else 'opt_clip_kernel')
            name = 'opt_sqsum@' + tag
        acc[name].append(float(r['Counter_Value']))
    return {k: (sum(v), len(v)) for k, v in acc.items()}


def main():
    fetch = per_kernel(sys.argv[1])
    write = per_kernel(sys.argv[2])
    out = {'_note': 'bytes per call; read = 2 * FETCH_SIZE(KB) * 1024 (gfx950 correction), '
                    'write = WRITE_SIZE(KB) * 1024'}
    out.update(library_stamp())
    for entry, kernels in GROUPS.items():
        rd = wr = 0.0
        found = []
        by_base = defaultdict(int)      # launches per kernel, template instances summed
        for kname in fetch:
            if any(k in kname for k in kernels):
                rd += 2 * fetch[kname][0] * 1024
                if 'opt_sqsum@' not in kname:
                    by_base[next(k for k in kernels if k in kname)] += fetch[kname][1]
                found.append(kname.replace('(anonymous namespace)::', '').split('(')[0])
        # one call launches one instance of each of its kernels (e.g. the 3x3
        # conv's relu / plain and edge forms, the stride-2 weight gradient's
        # four tilings): instances add up, distinct kernels of a call do not
        calls = (sum(by_base.values()) if entry in SUM_CALLS
                 else max(by_base.values(), default=0))
        for kname in write:
            if any(k in kname for k in kernels):
                wr += write[kname][0] * 1024
        # per call of the entry point = launches of its most frequent kernel
        # (the SN refresh skips P1 after a fused update: P1's bytes are spread
        # over the calls that did run it and those that did not)
        if found and calls:
            rd /= calls
            wr /= calls
            out[entry] = {'read_bytes': round(rd), 'write_bytes': round(wr),
                          'traffic_bytes': round(rd + wr), 'calls': calls,
                          'kernels': sorted(set(found))}
    print(json.dumps(out, indent=1))
    if len(sys.argv) > 3:
        with open(sys.argv[3], 'w') as f:
            json.dump(out, f, indent=1)


if __name__ == '__main__':
    main()
