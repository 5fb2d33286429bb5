# A/B of an environment switch on the bench, interleaved: bash tools/gpu_ab_env.sh TAG VAR "pytest -k expr"
set -o pipefail
TAG=${1:-abenv}
VAR=${2:-SMMD_RELU_POOL}
K=${3:-}
mkdir -p gpurun_out
export TMPDIR=/tmp
if [ -n "$K" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -k "$K" --timeout 300 --timeout-method thread > gpurun_out/${TAG}_tests.txt 2>&1 || { echo "tests rc=$?"; tail -40 gpurun_out/${TAG}_tests.txt; exit 1; }
  tail -2 gpurun_out/${TAG}_tests.txt
fi
for r in 1 2; do
  for v in 0 1; do
    env $VAR=$v timeout -k 10 600 python bench.py --steps 30 --warmup 6 --no-cpu-baseline --mmd-sweep 0 --ref-schedule-steps 0 > gpurun_out/${TAG}_${v}_${r}.json 2> gpurun_out/${TAG}_${v}_${r}.err || { echo "bench $v rc=$?"; tail -20 gpurun_out/${TAG}_${v}_${r}.err; exit 1; }
    python -c "import json; r=json.load(open('gpurun_out/${TAG}_${v}_${r}.json')); print('$VAR=$v run $r', r['value'], r['ms_per_step'], r['step_ms_by_kind'])"
  done
done
echo done
