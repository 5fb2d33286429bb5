# Round-4 baseline on a fresh box: the driver's bench command (no CPU leg) and
# a kernel trace of two whole 5D+1G cycles.  bash tools/gpu_baseline_r4.sh TAG
set -o pipefail
TAG=${1:-r4base}
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --mmd-sweep 0 --ref-schedule-steps 0 > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err || { echo "bench rc=$?"; tail -20 gpurun_out/${TAG}_bench.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/${TAG}_bench.json'));print(d['value'],d['ms_per_step'],d['step_ms_by_kind'])"
timeout -s KILL 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_trace -o run -- python tools/step_cycle.py --cycles 2 > gpurun_out/${TAG}_trace.log 2>&1 || { echo "trace rc=$?"; tail -5 gpurun_out/${TAG}_trace.log; exit 1; }
find gpurun_out/${TAG}_trace -name "*kernel_trace.csv" -exec gzip -f {} \;
echo done
