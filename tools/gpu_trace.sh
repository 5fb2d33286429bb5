# Kernel trace of a short bench run (timed region located by the step count):
# bash tools/gpu_trace.sh TAG [bench args]
set -o pipefail
TAG=${1:-trace}
shift
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace -d gpurun_out/${TAG} -o run --output-format csv -- python bench.py --no-cpu-baseline --mmd-sweep 0 --ref-schedule-steps 0 "$@" > gpurun_out/${TAG}.json 2> gpurun_out/${TAG}.err || { echo "trace rc=$?"; tail -20 gpurun_out/${TAG}.err; exit 1; }
f=$(find gpurun_out/${TAG} -name '*kernel_trace.csv' | head -1)
gzip -c "$f" > gpurun_out/${TAG}_kernel_trace.csv.gz
rm -f "$f"
head -c 400 gpurun_out/${TAG}.json
echo done
