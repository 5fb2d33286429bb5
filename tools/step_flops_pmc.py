"""Executed FLOPs and GPU time per kernel class over the last N steps of a
tools/step_cycle.py run (tools/gpu_step_pmc.sh): the counter-based step
roofline of SURVEY 8d beside bench.py's literal-MAC work-rate.

    python tools/step_flops_pmc.py PMC_DIR TRACE_DIR [steps [PMC2_DIR]]

FLOPs per dispatch (fp32, wave64; rocprofv3 counts wave-instructions):
  512 * SQ_INSTS_VALU_MFMA_MOPS_F32   (MFMA, in units of 512 flops)
+ 128 * SQ_INSTS_VALU_FMA_F32         (64 lanes x 2)
+  64 * (SQ_INSTS_VALU_ADD_F32 + SQ_INSTS_VALU_MUL_F32 + SQ_INSTS_VALU_TRANS_F32)
PMC2_DIR (optional): a pass with the hardware FLOP tallies
SQ_INSTS_VALU_FLOPS_FP32 (+ _TRANS).  On gfx950 they tally per wave (x 64
lanes gives the flops: 5.53 x 64 = 354 GFLOP per step on the Winograd
kernels, the instruction-count figure above to 0.1 %), so packed (v_pk_*)
operations would show as a difference between the two; reported per class
as `hw_valu_gflop_per_step` and `hw_tflops` = (64 x tally + MFMA) / time.
The window: every step ends in one optimizer update kernel (opt_adam*), so
the last `steps` steps are the dispatches after the (updates - steps)-th one.
"""
import collections
import csv
import glob
import gzip
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from stamp import library_stamp  # noqa: E402

FP32_PEAK_TFS = 157.3


def _open(path):
    return gzip.open(path, 'rt') if path.endswith('.gz') else open(path)


def _find(d, name):
    fs = glob.glob(os.path.join(d, '**', '*' + name + '*'), recursive=True)
    if not fs:
        raise SystemExit('no %s under %s' % (name, d))
    return sorted(fs)[0]


def kclass(k):
    if 'Sp3Asm' in k or 'inograd' in k:
        return 'miopen_winograd'
    if 'smmd::' in k and 'wino_wgrad' in k:
        return 'smmd_wino3x3_wgrad'
    if 'smmd::' in k and ('wino_' in k):
        return 'smmd_wino3x3'
    if 'smmd::' in k and ('s2_' in k or 's2t_' in k):
        return 'smmd_wino_s2'
    for key, c in (('igemm_wrw', 'igemm_wrw'), ('igemm_bwd', 'igemm_bwd'),
                   ('igemm_fwd', 'igemm_fwd'), ('ransform', 'miopen_transform'),
                   ('transpose', 'transpose'), ('smmd::', 'smmd_library'),
                   ('Cijk', 'hipblaslt_gemm'), ('BatchNorm', 'batchnorm'),
                   ('TensorOp', 'miopen_tensorop'), ('at::native', 'torch_elementwise')):
        if key in k:
            return c
    return 'other'


def window(rows, steps):
    """rows sorted by dispatch order -> the rows of the last `steps` steps."""
    ups = [i for i, r in enumerate(rows) if 'opt_adam' in r['name']]
    if len(ups) < steps + 1:
        raise SystemExit('only %d update kernels' % len(ups))
    a = ups[len(ups) - steps - 1]
    return rows[a + 1:ups[-1] + 1]


def load_pmc(d):
    path = _find(d, 'counter_collection.csv')
    disp = collections.OrderedDict()
    for r in csv.DictReader(_open(path)):
        key = int(r.get('Dispatch_Id') or r.get('Correlation_Id'))
        e = disp.setdefault(key, {'name': r['Kernel_Name'], 'c': {}})
        e['c'][r['Counter_Name']] = e['c'].get(r['Counter_Name'], 0.0) + float(r['Counter_Value'])
    return [dict(id=k, **v) for k, v in sorted(disp.items())]


def load_trace(d):
    path = _find(d, 'kernel_trace.csv')
    rows = [{'name': r['Kernel_Name'], 's': int(r['Start_Timestamp']),
             'e': int(r['End_Timestamp'])} for r in csv.DictReader(_open(path))]
    rows.sort(key=lambda r: r['s'])
    return rows


def flops(c):
    return (512.0 * c.get('SQ_INSTS_VALU_MFMA_MOPS_F32', 0.0)
            + 128.0 * c.get('SQ_INSTS_VALU_FMA_F32', 0.0)
            + 64.0 * (c.get('SQ_INSTS_VALU_ADD_F32', 0.0) + c.get('SQ_INSTS_VALU_MUL_F32', 0.0)
                      + c.get('SQ_INSTS_VALU_TRANS_F32', 0.0)))


def main():
    pmc_dir, trace_dir = sys.argv[1], sys.argv[2]
    steps = int(sys.argv[3]) if len(sys.argv) > 3 else 12
    pw = window(load_pmc(pmc_dir), steps)
    hw = collections.Counter()
    if len(sys.argv) > 4:
        for r in window(load_pmc(sys.argv[4]), steps):
            c = r['c']
            hw[kclass(r['name'])] += 64.0 * (c.get('SQ_INSTS_VALU_FLOPS_FP32', 0.0)
                                             + c.get('SQ_INSTS_VALU_FLOPS_FP32_TRANS', 0.0))
    tw = window(load_trace(trace_dir), steps)
    fl = collections.Counter()
    mf = collections.Counter()
    n = collections.Counter()
    for r in pw:
        k = kclass(r['name'])
        fl[k] += flops(r['c'])
        mf[k] += 512.0 * r['c'].get('SQ_INSTS_VALU_MFMA_MOPS_F32', 0.0)
        n[k] += 1
    t = collections.Counter()
    for r in tw:
        t[kclass(r['name'])] += (r['e'] - r['s']) * 1e-9
    busy = sum(t.values())
    out = {'steps': steps, 'dispatches': len(pw), 'trace_dispatches': len(tw),
           'gpu_busy_ms_per_step': round(busy / steps * 1e3, 3),
           'executed_tflop_per_step': round(sum(fl.values()) / steps / 1e12, 4),
           'executed_tflops_over_busy': round(sum(fl.values()) / busy / 1e12, 2),
           'frac_of_fp32_peak_over_busy': round(sum(fl.values()) / busy / 1e12 / FP32_PEAK_TFS, 4),
           'classes': {}}
    out.update(library_stamp())
    if hw:
        tot = sum(hw.values()) + sum(mf.values())
        out.update(hw_executed_tflop_per_step=round(tot / steps / 1e12, 4),
                   hw_executed_tflops_over_busy=round(tot / busy / 1e12, 2),
                   hw_frac_of_fp32_peak_over_busy=round(tot / busy / 1e12 / FP32_PEAK_TFS, 4))
    for k in sorted(set(fl) | set(t), key=lambda k: -t.get(k, 0)):
        tk = t.get(k, 0.0)
        out['classes'][k] = {
            'dispatches_per_step': round(n[k] / steps, 1),
            'ms_per_step': round(tk / steps * 1e3, 3),
            'time_frac': round(tk / busy, 4) if busy else None,
            'executed_gflop_per_step': round(fl[k] / steps / 1e9, 2),
            'mfma_gflop_per_step': round(mf[k] / steps / 1e9, 2),
            'executed_flop_frac': round(fl[k] / max(sum(fl.values()), 1.0), 4),
            'tflops': round(fl[k] / tk / 1e12, 2) if tk else None,
            'frac_of_fp32_peak': round(fl[k] / tk / 1e12 / FP32_PEAK_TFS, 4) if tk else None}
        if hw:
            fk = hw[k] + mf[k]
            out['classes'][k].update(
                hw_valu_gflop_per_step=round(hw[k] / steps / 1e9, 2),
                hw_tflops=round(fk / tk / 1e12, 2) if tk else None,
                hw_frac_of_fp32_peak=round(fk / tk / 1e12 / FP32_PEAK_TFS, 4) if tk else None)
    print(json.dumps(out, indent=1))


if __name__ == '__main__':
    main()
