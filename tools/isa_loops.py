"""Instruction mix of the MFMA loops of the library's kernels, from the
compiler's gfx950 assembly (no GPU needed):

    python tools/isa_loops.py scaled-mmd-gan_amd/csrc/smmd_wino_wgrad.hip [kernel-substring]

For every loop (a backward branch) that contains MFMAs and no inner loop with
MFMAs: MFMA, VALU (and the v_mov / v_xor among them), SALU, LDS reads / writes,
vector memory, waitcnt, barriers -- per loop iteration and per MFMA.  In an f32
MFMA kernel every VALU instruction costs SIMD time beside the MFMA
(profiles/r12/mfma_valu_coissue.txt), so VALU per MFMA is the number to cut."""
import collections
import os
import re
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def assemble(src, defs=()):
    out = os.path.join(tempfile.mkdtemp(), 'k.s')
    cmd = ['/opt/rocm/bin/hipcc', '--offload-arch=gfx950', '-O3', '-std=c++17',
           '-I' + os.path.join(ROOT, 'include'), '--cuda-device-only', '-S', src, '-o', out]
    subprocess.run(cmd + list(defs), check=True, capture_output=True)
    return open(out).read().split('\n')


def kernels(lines):
    starts = [(i, l.split(':')[0]) for i, l in enumerate(lines)
              if re.match(r'^_Z\S+:', l) or re.match(r'^[a-zA-Z_]\w*:\s*(;.*)?$', l)]
    for j, (i, name) in enumerate(starts):
        end = starts[j + 1][0] if j + 1 < len(starts) else len(lines)
        yield name, lines[i:end]


def classify(seg):
    c = collections.Counter()
    for l in seg:
        l = l.strip()
        if not l or l[0] in ';.':
            continue
        op = l.split()[0]
        if op.startswith('v_mfma'):
            c['mfma'] += 1
        elif op.startswith('v_'):
            c['valu'] += 1
            if op.startswith(('v_mov', 'v_pk_mov')):
                c['v_mov'] += 1
            if op.startswith('v_xor'):
                c['v_xor'] += 1
            if op.startswith(('v_add_u32', 'v_add3_u32', 'v_lshl', 'v_mad_u', 'v_mul_lo', 'v_mul_u32',
                              'v_and_b32', 'v_or_b32', 'v_lshr', 'v_sub_u32', 'v_ashr')):
                c['v_int'] += 1
        elif op.startswith('s_waitcnt'):
            c['wait'] += 1
        elif op.startswith('s_barrier'):
            c['barrier'] += 1
        elif op.startswith('s_'):
            c['salu'] += 1
        elif op.startswith(('ds_read', 'ds_load')):
            c['lds_r'] += 1
        elif op.startswith(('ds_write', 'ds_store')):
            c['lds_w'] += 1
        elif op.startswith(('buffer_', 'global_')):
            c['vmem'] += 1
    return c


def main():
    src = sys.argv[1]
    want = sys.argv[2] if len(sys.argv) > 2 else ''
    defs = sys.argv[3:]
    lines = assemble(src, defs)
    for name, body in kernels(lines):
        if want not in name or 'mfma' not in '\n'.join(body):
            continue
        labels = {m.group(1): i for i, l in enumerate(body)
                  for m in [re.match(r'^(\.LBB\S+):', l)] if m}
        loops = []
        for i, l in enumerate(body):
            m = re.search(r's_(?:cbranch_\w+|branch)\s+(\.LBB\S+)', l)
            if m and m.group(1) in labels and labels[m.group(1)] < i:
                loops.append((labels[m.group(1)], i))
        loops = [(a, b) for a, b in loops if classify(body[a:b + 1])['mfma'] > 0]
        inner = [(a, b) for a, b in loops
                 if not any(a < a2 and b2 <= b and (a2, b2) != (a, b) for a2, b2 in loops)]
        print(name[:110])
        for a, b in inner:
            c = classify(body[a:b + 1])
            m = c['mfma']
            print('  loop %5d-%5d: ' % (a, b) +
                  ' '.join('%s %d' % (k, c[k]) for k in ('mfma', 'valu', 'v_mov', 'v_xor', 'v_int',
                                                         'salu', 'lds_r', 'lds_w', 'vmem', 'wait',
                                                         'barrier')) +
                  '   per MFMA: valu %.2f v_mov %.2f salu %.2f lds %.2f' % (
                      c['valu'] / m, c['v_mov'] / m, c['salu'] / m, (c['lds_r'] + c['lds_w']) / m))


if __name__ == '__main__':
    main()
