"""Per-kernel summary of a rocprofv3 SQLite output (the default format):
    python tools/prof_db.py DIR_OR_DB [N]
name, calls, mean / min / max duration (us), share of the total."""
import glob
import os
import sqlite3
import sys


def main():
    p = sys.argv[1]
    n = int(sys.argv[2]) if len(sys.argv) > 2 else 30
    f = p if p.endswith('.db') else glob.glob(os.path.join(p, '**', '*.db'), recursive=True)[0]
    c = sqlite3.connect(f)
    rows = list(c.execute('select name, count(*), avg(duration), min(duration), max(duration), '
                          'sum(duration) from kernels group by name order by sum(duration) desc'))
    tot = sum(r[5] for r in rows)
    print('%7s %9s %9s %9s %7s  %s' % ('calls', 'mean_us', 'min_us', 'max_us', 'share', 'kernel'))
    for r in rows[:n]:
        print('%7d %9.2f %9.2f %9.2f %6.2f%%  %s' % (r[1], r[2] / 1e3, r[3] / 1e3, r[4] / 1e3,
                                                     100 * r[5] / tot, r[0][:110]))


if __name__ == '__main__':
    main()
