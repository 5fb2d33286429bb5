# Full GPU check of the tree: every gpu test, the driver's bench command, and a
# kernel trace of two whole 5D+1G cycles.  bash tools/gpu_round.sh TAG [skip_tests]
set -o pipefail
TAG=${1:-round}
mkdir -p gpurun_out
export TMPDIR=/tmp
if [ "${2:-0}" != "1" ]; then
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/${TAG}_tests.txt 2>&1 || { echo "tests rc=$?"; tail -30 gpurun_out/${TAG}_tests.txt; exit 1; }
tail -1 gpurun_out/${TAG}_tests.txt
fi
timeout -k 10 400 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --mmd-sweep 0 --ref-schedule-steps 0 > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err || { echo "bench rc=$?"; tail -20 gpurun_out/${TAG}_bench.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/${TAG}_bench.json'));print(d['value'],d['ms_per_step'],d['step_ms_by_kind'],d['roofline']['kernel'],d['roofline']['frac'])"
timeout -s KILL 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_trace -o run -- python tools/step_cycle.py --cycles 2 > gpurun_out/${TAG}_trace.log 2>&1 || { echo "trace rc=$?"; tail -5 gpurun_out/${TAG}_trace.log; exit 1; }
find gpurun_out/${TAG}_trace -name "*kernel_trace.csv" -exec gzip -f {} \;
find gpurun_out/${TAG}_trace -name '*kernel_stats.csv' -exec head -16 {} \; | cut -c1-150
echo done
