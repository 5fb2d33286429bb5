# rocprof kernel stats of tools/thin_bench.py: bash tools/gpu_thinprof.sh TAG
set -o pipefail
TAG=${1:-thinprof}
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG} -o run -- python tools/thin_bench.py 50 > gpurun_out/${TAG}.log 2>&1 || { echo "rc=$?"; tail -20 gpurun_out/${TAG}.log; exit 1; }
cat gpurun_out/${TAG}.log | grep us/call
S=$(find gpurun_out/${TAG} -name '*kernel_stats.csv' | head -1)
python - "$S" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
for r in sorted(rows, key=lambda r: -float(r['TotalDurationNs']))[:25]:
    print('%-90s %6s calls %9.1f us avg' % (r['Name'][:90], r['Calls'], float(r['AverageNs']) / 1e3))
PY
