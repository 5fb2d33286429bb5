"""Per-step GPU time by kernel class and the top elementwise kernels over a
window of whole steps of a bench kernel trace (tools/gpu_trace.sh output).

    python tools/trace_window.py gpurun_out/TAG_kernel_trace.csv.gz [first_adam] [n_steps]
"""
import collections
import csv
import gzip
import re
import sys


def main():
    path = sys.argv[1]
    a0 = int(sys.argv[2]) if len(sys.argv) > 2 else 10
    n = int(sys.argv[3]) if len(sys.argv) > 3 else 12
    op = gzip.open if path.endswith('.gz') else open
    rows = sorted(csv.DictReader(op(path, 'rt')), key=lambda r: int(r['Start_Timestamp']))
    adams = [i for i, r in enumerate(rows) if 'opt_adam' in r['Kernel_Name']]
    a, b = adams[a0], adams[a0 + n]
    ws, we = int(rows[a]['End_Timestamp']), int(rows[b]['End_Timestamp'])
    cat = collections.Counter()
    elt = collections.defaultdict(lambda: [0, 0])
    busy, cur = 0, ws
    for r in rows[a + 1:b + 1]:
        s, e = int(r['Start_Timestamp']), int(r['End_Timestamp'])
        busy += max(0, e - max(s, cur))
        cur = max(cur, e)
        k = r['Kernel_Name']
        c = ('winograd' if 'Sp3Asm' in k else 'igemm_wrw' if 'igemm_wrw' in k else
             'igemm_bwd' if 'igemm_bwd' in k else 'igemm_fwd' if 'igemm_fwd' in k else
             'transpose' if 'transpose' in k else 'smmd' if 'smmd' in k else
             'gemm(Cijk)' if 'Cijk' in k else 'batchnorm' if 'BatchNorm' in k else
             'miopen_tensorop' if 'TensorOp' in k else 'torch_elementwise' if 'at::native' in k
             else k[:40])
        cat[c] += e - s
        if c in ('torch_elementwise', 'smmd'):
            m = re.search(r'(smmd::\w+|at::native::(?:\(anonymous namespace\)::)?\w+)', k)
            f = re.findall(r'(CUDAFunctor_\w+|threshold|leaky_relu\w*|clamp\w*|FillFunctor|'
                           r'MulFunctor|upsample\w*|avg_pool\w*|sigmoid\w*|BinaryFunctor)', k)
            key = (m.group(1) if m else k[:40]) + ' ' + ' '.join(dict.fromkeys(f))
            elt[(key[:80], r['Grid_Size_X'])][0] += e - s
            elt[(key[:80], r['Grid_Size_X'])][1] += 1
    span = we - ws
    print('%d steps: %.3f ms/step, GPU busy %.1f%%' % (n, span / n / 1e6, 100 * busy / span))
    for k, v in cat.most_common():
        print('  %-24s %7.3f ms/step %5.1f%%' % (k, v / n / 1e6, 100 * v / span))
    print('top elementwise / library kernels:')
    for (k, g), (t, c) in sorted(elt.items(), key=lambda kv: -kv[1][0])[:30]:
        print('  %7.1f us/step %5.1f calls/step %7.1f us grid %9s  %s' % (t / n / 1e3, c / n,
                                                                        t / c / 1e3, g, k))


if __name__ == '__main__':
    main()
