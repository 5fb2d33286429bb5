# Kernel trace (+ stats) of whole 5D+1G cycles of the bench workload and the
# per-kernel library durations: bash tools/gpu_trace_cycle.sh TAG [step_cycle args]
set -o pipefail
TAG=${1:-trace}
shift
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -s KILL 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_trace -o run -- python tools/step_cycle.py "$@" > gpurun_out/${TAG}_trace.log 2>&1 || { echo "trace rc=$?"; tail -5 gpurun_out/${TAG}_trace.log; exit 1; }
f=$(find gpurun_out/${TAG}_trace -name "*kernel_trace.csv" | head -1)
python tools/trace_by_grid.py $f smmd:: > gpurun_out/${TAG}_smmd_kernels.txt
gzip -f $f
cat gpurun_out/${TAG}_smmd_kernels.txt
