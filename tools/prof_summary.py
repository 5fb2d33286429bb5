"""Summarise a rocprofv3 kernel_stats.csv: python tools/prof_summary.py <csv> [filter]"""
import csv
import sys
rows = list(csv.DictReader(open(sys.argv[1])))
flt = sys.argv[2] if len(sys.argv) > 2 else None
tot = sum(float(r['TotalDurationNs']) for r in rows)
print('total kernel ms %.1f' % (tot / 1e6))
for r in sorted(rows, key=lambda r: -float(r['TotalDurationNs'])):
    if flt and flt not in r['Name']:
        continue
    print('%6.2f%% n=%5s avg=%9.2fus min=%9.2fus  %s' % (100 * float(r['TotalDurationNs']) / tot, r['Calls'],
          float(r['AverageNs']) / 1e3, float(r['MinNs']) / 1e3, r['Name'][:100]))
