# Winograd kernels after a change: their GPU tests and standalone timing
set -o pipefail
TAG=${1:-xcd}
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_wino.py tests/test_gpu_wino_s2.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/${TAG}_tests.txt 2>&1 || { echo "tests rc=$?"; tail -30 gpurun_out/${TAG}_tests.txt; exit 1; }
tail -1 gpurun_out/${TAG}_tests.txt
timeout -k 10 200 python -u tools/wino_bench.py --iters 20 > gpurun_out/${TAG}_w3.txt 2>&1 || { echo "w3 rc=$?"; exit 1; }
grep '^{' gpurun_out/${TAG}_w3.txt | python -c "import sys,json; [print(r['shape'], round(r['wino_us'],1), 'miopen', round(r['miopen_fwd_us'],1)) for r in map(json.loads, sys.stdin)]"
timeout -k 10 200 python -u tools/wino_s2_bench.py > gpurun_out/${TAG}_s2.txt 2>&1 || { echo "s2 rc=$?"; exit 1; }
grep '^{' gpurun_out/${TAG}_s2.txt | python -c "import sys,json; [print(r['shape'], r['wino_us'], r['dgrad_wino_us']) for r in map(json.loads, sys.stdin)]"
