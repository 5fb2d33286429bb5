# thin-conv pass: its GPU tests, then an A/B bench (library thin kernels vs MIOpen)
# usage: bash tools/gpu_thin.sh TAG
set -o pipefail
TAG=${1:-thin}
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_thin.py -x -q --timeout 300 --timeout-method thread > gpurun_out/${TAG}_tests.txt 2>&1 || { echo "tests rc=$?"; tail -40 gpurun_out/${TAG}_tests.txt; exit 1; }
tail -2 gpurun_out/${TAG}_tests.txt
for T in 1 0; do
  SMMD_THIN_CONV=$T timeout -k 10 400 python bench.py --steps 30 --warmup 6 --no-cpu-baseline --mmd-sweep 0 --ref-schedule-steps 0 > gpurun_out/${TAG}_bench_t$T.json 2> gpurun_out/${TAG}_bench_t$T.err || { echo "bench rc=$?"; tail -20 gpurun_out/${TAG}_bench_t$T.err; exit 1; }
  python - <<PY
import json
r = json.load(open('gpurun_out/${TAG}_bench_t$T.json'))
print('thin=$T value', r['value'], 'ms/step', r['ms_per_step'], r['step_ms_by_kind'])
for k, v in r['hip_kernels'].items():
    if 'thin' in k: print(' ', k, v)
PY
done
echo done
