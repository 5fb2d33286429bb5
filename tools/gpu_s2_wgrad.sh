# Stride-2 Winograd weight gradient: parity tests, timing vs MIOpen, rocprof
# kernel split.  bash tools/gpu_s2_wgrad.sh TAG
set -o pipefail
TAG=${1:-s2w}
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_wino_s2.py -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/${TAG}_tests.txt 2>&1 || { echo "tests rc=$?"; tail -30 gpurun_out/${TAG}_tests.txt; exit 1; }
tail -1 gpurun_out/${TAG}_tests.txt
timeout -k 10 300 python -u tools/s2_wgrad_bench.py > gpurun_out/${TAG}_bench.txt 2>&1 || { echo "bench rc=$?"; tail -20 gpurun_out/${TAG}_bench.txt; exit 1; }
cat gpurun_out/${TAG}_bench.txt
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_prof -o run -- python tools/s2_wgrad_bench.py --iters 5 > gpurun_out/${TAG}_prof.log 2>&1 || { echo "prof rc=$?"; tail -5 gpurun_out/${TAG}_prof.log; exit 1; }
find gpurun_out/${TAG}_prof -name '*kernel_stats.csv' -exec head -12 {} \; | cut -c1-180
