# quick GPU pass: the GPU tests, then a short bench line with the MMD sweep
# usage: bash tools/gpu_quick.sh TAG [pytest -k expr]
set -o pipefail
TAG=${1:-quick}
K=${2:-}
mkdir -p gpurun_out
export TMPDIR=/tmp
if [ -n "$K" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -k "$K" --timeout 300 --timeout-method thread > gpurun_out/${TAG}_tests.txt 2>&1 || { echo "tests rc=$?"; tail -40 gpurun_out/${TAG}_tests.txt; exit 1; }
else
  timeout -k 10 1200 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/${TAG}_tests.txt 2>&1 || { echo "tests rc=$?"; tail -40 gpurun_out/${TAG}_tests.txt; exit 1; }
fi
tail -2 gpurun_out/${TAG}_tests.txt
timeout -k 10 600 python bench.py --steps 30 --warmup 6 --no-cpu-baseline --mmd-sweep 2 > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err || { echo "bench rc=$?"; tail -20 gpurun_out/${TAG}_bench.err; exit 1; }
python - <<PY
import json
r = json.load(open('gpurun_out/${TAG}_bench.json'))
print('value', r['value'], 'ms/step', r['ms_per_step'])
for row in r['mmd_sweep']:
    print(row['kernel'], row['N'], row['D'], 'kernel_ms', row['kernel_ms'], 'valu', row.get('valu_frac'), 'op_ms', row['op_ms'])
print('mmd in step', r['roofline_hot_path'].get('smmd_mmd2_fwd'))
PY
echo done
