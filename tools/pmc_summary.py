"""Per-kernel means of rocprofv3 counter passes.
    python tools/pmc_summary.py DIR [DIR ...] SUBSTRING
Prints, per kernel name containing SUBSTRING (and grid size), the mean of
every counter over its dispatches, plus the derived MFMA busy fraction
(SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE x 1024 SIMDs... reported raw)."""
import collections
import csv
import glob
import gzip
import os
import sys


def main():
    dirs, sub = sys.argv[1:-1], sys.argv[-1]
    acc = collections.defaultdict(lambda: collections.defaultdict(list))
    for d in dirs:
        for path in glob.glob(os.path.join(d, '**', '*counter_collection.csv*'), recursive=True):
            disp = collections.defaultdict(dict)
            fh = gzip.open(path, 'rt') if path.endswith('.gz') else open(path)
            for r in csv.DictReader(fh):
                if sub not in r['Kernel_Name']:
                    continue
                key = (r['Kernel_Name'].replace('(anonymous namespace)::', '').split('(')[0],
                       r.get('Grid_Size', ''))
                disp[(key, r['Dispatch_Id'])][r['Counter_Name']] = (
                    disp[(key, r['Dispatch_Id'])].get(r['Counter_Name'], 0.0)
                    + float(r['Counter_Value']))
            for (key, _), cs in disp.items():
                for c, v in cs.items():
                    acc[key][c].append(v)
    for key in sorted(acc):
        cs = acc[key]
        print(key[0], 'grid', key[1])
        for c in sorted(cs):
            vs = cs[c]
            print('   %-30s %14.4g  (n=%d)' % (c, sum(vs) / len(vs), len(vs)))


if __name__ == '__main__':
    main()
