# MMD kernel microbench: tiled vs row-sweep path, and a rocprofv3 kernel trace
set -o pipefail
TAG=${1:-mmdb}
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python tools/mmd_bench.py --json gpurun_out/${TAG}_tile.json || exit 1
SMMD_MMD_TILE=0 timeout -k 10 300 python tools/mmd_bench.py --grid rbf:64:1,rbf:512:1,rbf:2048:1 --json gpurun_out/${TAG}_sweep.json || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${TAG}_prof -o run --output-format csv -- python tools/mmd_bench.py --iters 20 > gpurun_out/${TAG}_prof.log 2>&1 || { echo "prof rc=$?"; tail gpurun_out/${TAG}_prof.log; exit 1; }
find gpurun_out/${TAG}_prof -name "*kernel_stats.csv" -exec cat {} \; | head -20
echo done
