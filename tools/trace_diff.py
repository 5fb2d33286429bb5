"""Per-kernel time of the last K steps of two kernel traces (rocprofv3
--kernel-trace csv.gz), a step ending at each optimizer launch (opt_adam*):
python tools/trace_diff.py A.csv.gz B.csv.gz [K]"""
import collections
import csv
import gzip
import re
import sys


def window(path, k):
    rows = sorted(csv.DictReader(gzip.open(path, 'rt')), key=lambda r: int(r['Start_Timestamp']))
    ends = [i for i, r in enumerate(rows) if re.search(r'opt_adam', r['Kernel_Name'])]
    lo = ends[-k - 1] + 1
    sel = rows[lo:ends[-1] + 1]
    t0, t1 = int(sel[0]['Start_Timestamp']), int(sel[-1]['End_Timestamp'])
    per = collections.defaultdict(lambda: [0, 0.0])
    busy = 0
    for r in sel:
        n = re.sub(r'\(.*', '', r['Kernel_Name'])[:70]
        d = (int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1e3
        per[n][0] += 1
        per[n][1] += d
        busy += d
    return per, (t1 - t0) / 1e3, busy, len(sel)


def main():
    a, b = sys.argv[1], sys.argv[2]
    k = int(sys.argv[3]) if len(sys.argv) > 3 else 12
    pa, wa, ba, na = window(a, k)
    pb, wb, bb, nb = window(b, k)
    print('A: %d launches, window %.1f us, busy %.1f us (%.1f us/step)' % (na, wa, ba, wa / k))
    print('B: %d launches, window %.1f us, busy %.1f us (%.1f us/step)' % (nb, wb, bb, wb / k))
    names = set(pa) | set(pb)
    diff = sorted(names, key=lambda n: -abs(pb.get(n, [0, 0])[1] - pa.get(n, [0, 0])[1]))
    print('%-70s %6s %6s %10s %10s' % ('kernel', 'nA', 'nB', 'usA/step', 'usB-usA'))
    for n in diff[:30]:
        ca, ta = pa.get(n, [0, 0.0])
        cb, tb = pb.get(n, [0, 0.0])
        print('%-70s %6d %6d %10.1f %10.1f' % (n, ca, cb, ta / k, (tb - ta) / k))


if __name__ == '__main__':
    main()
