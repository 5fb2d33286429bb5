set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/lin -o run --output-format csv -- python tools/linear_bench.py > gpurun_out/lin.log 2>&1 || { echo "rc=$?"; tail -20 gpurun_out/lin.log; exit 1; }
f=$(find gpurun_out/lin -name '*kernel_trace.csv' | head -1)
python - "$f" <<'PY'
import csv, sys
rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r['Start_Timestamp']))
segs, cur = [], [rows[0]]
for a, b in zip(rows, rows[1:]):
    if int(b['Start_Timestamp']) - int(a['End_Timestamp']) > 20e6:
        segs.append(cur); cur = []
    cur.append(b)
segs.append(cur)
for i, s in enumerate(segs):
    tot = sum(int(r['End_Timestamp']) - int(r['Start_Timestamp']) for r in s)
    names = {}
    for r in s:
        n = r['Kernel_Name'][:50]
        names[n] = names.get(n, 0) + int(r['End_Timestamp']) - int(r['Start_Timestamp'])
    top = sorted(names.items(), key=lambda kv: -kv[1])[:4]
    print('seg %2d kernels %6d kernel-us %9.1f  top %s' % (i, len(s), tot / 1e3, [(n, round(t / 1e3)) for n, t in top]))
PY
cat gpurun_out/lin.log | grep M=
