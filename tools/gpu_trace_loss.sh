# Kernel durations of the loss side alone: bash tools/gpu_trace_loss.sh TAG
set -o pipefail
TAG=${1:-loss}
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -s KILL 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_trace -o run -- python tools/loss_bench.py --iters 200 > gpurun_out/${TAG}.log 2>&1 || { echo "trace rc=$?"; tail -5 gpurun_out/${TAG}.log; exit 1; }
f=$(find gpurun_out/${TAG}_trace -name "*kernel_trace.csv" | head -1)
python tools/trace_by_grid.py $f smmd:: | tee gpurun_out/${TAG}_kernels.txt
gzip -f $f
