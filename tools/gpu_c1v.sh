# 1x1 kernel variants A/B (tools/c1_probe.py over tools/hip/c1_*.so) and the
# stamped library.  bash tools/gpu_c1v.sh TAG LIBS
set -o pipefail
TAG=${1:-c1v}
LIBS=${2:-c1_base}
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u tools/c1_probe.py --libs $LIBS > gpurun_out/${TAG}.txt 2>&1 || { echo "probe rc=$?"; tail -20 gpurun_out/${TAG}.txt; exit 1; }
grep -v "^{" gpurun_out/${TAG}.txt || true
if [ -n "$3" ]; then
  timeout -s KILL 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_tr -o run -- python tools/c1_probe.py --libs $3 --iters 20 > gpurun_out/${TAG}_tr.log 2>&1 || { echo "trace rc=$?"; tail -5 gpurun_out/${TAG}_tr.log; exit 1; }
fi
