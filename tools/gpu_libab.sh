# Library A/B on one box: tools/hipbench.py with a baseline libsmmd_hip.so
# (ab/libsmmd_base.so, built from an earlier commit) and with the tree's own,
# interleaved, then the GPU tests of the touched kernels.
# usage: bash tools/gpu_libab.sh TAG ["pytest -k expr"]
set -o pipefail
TAG=${1:-libab}
K=${2:-}
mkdir -p gpurun_out
export TMPDIR=/tmp
for r in 1 2; do
  for v in base new; do
    if [ "$v" = base ]; then export SMMD_HIP_LIB=$PWD/ab/libsmmd_base.so; else unset SMMD_HIP_LIB; fi
    timeout -k 10 300 python tools/hipbench.py --json gpurun_out/${TAG}_${v}${r}.json > gpurun_out/${TAG}_${v}${r}.log 2>&1 || { echo "hipbench $v rc=$?"; tail -20 gpurun_out/${TAG}_${v}${r}.log; exit 1; }
  done
done
unset SMMD_HIP_LIB
python - <<PY
import json
for r in (1, 2):
    a = json.load(open('gpurun_out/${TAG}_base%d.json' % r))
    b = json.load(open('gpurun_out/${TAG}_new%d.json' % r))
    for k in a:
        if k in b:
            print('%d %-34s base %8.2f us  new %8.2f us  frac %s -> %s' % (
                r, k, a[k]['avg_us'], b[k]['avg_us'], a[k].get('frac'), b[k].get('frac')))
PY
if [ "$PROF" = 1 ]; then
  for v in base new; do
    if [ "$v" = base ]; then export SMMD_HIP_LIB=$PWD/ab/libsmmd_base.so; else unset SMMD_HIP_LIB; fi
    timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${TAG}_prof_$v -o run --output-format csv -- python tools/hipbench.py --iters 100 > gpurun_out/${TAG}_prof_$v.log 2>&1 || { echo "prof $v rc=$?"; tail -20 gpurun_out/${TAG}_prof_$v.log; exit 1; }
  done
  unset SMMD_HIP_LIB
  for v in base new; do
    echo "== $v"
    f=$(find gpurun_out/${TAG}_prof_$v -name '*kernel_stats.csv' | head -1)
    python - "$f" <<'PY2'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    if 'smmd::' in r['Name']:
        print('%-60s %6s calls  avg %8.2f us' % (r['Name'][:60], r['Calls'], float(r['AverageNs']) / 1e3))
PY2
  done
fi
if [ -n "$K" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -k "$K" --timeout 300 --timeout-method thread > gpurun_out/${TAG}_tests.txt 2>&1 || { echo "tests rc=$?"; tail -40 gpurun_out/${TAG}_tests.txt; exit 1; }
  tail -2 gpurun_out/${TAG}_tests.txt
fi
echo done
