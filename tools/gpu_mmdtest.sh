# MMD parity tests + microbench (tiled vs row sweep)
set -o pipefail
TAG=${1:-mmdt}
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py -x -q -k "mmd2" --timeout 300 --timeout-method thread > gpurun_out/${TAG}_tests.txt 2>&1 || { echo "tests rc=$?"; tail -40 gpurun_out/${TAG}_tests.txt; exit 1; }
tail -2 gpurun_out/${TAG}_tests.txt
timeout -k 10 300 python tools/mmd_bench.py --json gpurun_out/${TAG}_tile.json || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${TAG}_prof -o run --output-format csv -- python tools/mmd_bench.py --iters 20 > gpurun_out/${TAG}_prof.log 2>&1 || { echo "prof rc=$?"; tail gpurun_out/${TAG}_prof.log; exit 1; }
find gpurun_out/${TAG}_prof -name "*kernel_stats.csv" -exec cat {} \; | head -12
echo done
