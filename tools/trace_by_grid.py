"""Mean kernel duration per (kernel, grid size) from a rocprofv3 kernel trace.

    python tools/trace_by_grid.py run_kernel_trace.csv [substring]
"""
import csv
import sys
from collections import defaultdict


def main():
    path = sys.argv[1]
    sub = sys.argv[2] if len(sys.argv) > 2 else 'smmd::'
    acc = defaultdict(list)
    for r in csv.DictReader(open(path)):
        name = r['Kernel_Name']
        if sub not in name:
            continue
        grid = r.get('Grid_Size_X') or r.get('Grid_Size') or '?'
        dur = (int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1e3
        acc[(name.split('(')[0][:70], grid)].append(dur)
    for (name, grid), v in sorted(acc.items()):
        v.sort()
        print('%-70s grid %8s  n %4d  mean %8.2f us  median %8.2f us' % (
            name, grid, len(v), sum(v) / len(v), v[len(v) // 2]))


if __name__ == '__main__':
    main()
