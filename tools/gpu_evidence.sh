# Round evidence, part A: the whole -m gpu suite, smoke(), the default bench
# (CPU baseline included).  Part B (tools/gpu_evidence_b.sh): the driver's
# command, a rocprof kernel trace + stats of the bench, the 2-rank launch, the
# batch-256 line.  bash tools/gpu_evidence.sh TAG
set -o pipefail
TAG=${1:-ev}
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/${TAG}_gpu_tests.txt 2>&1 || { echo "tests rc=$?"; tail -40 gpurun_out/${TAG}_gpu_tests.txt; exit 1; }
tail -2 gpurun_out/${TAG}_gpu_tests.txt
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${TAG}_smoke.txt 2>&1 || { echo "smoke rc=$?"; tail -20 gpurun_out/${TAG}_smoke.txt; exit 1; }
tail -1 gpurun_out/${TAG}_smoke.txt
timeout -k 10 900 python bench.py > gpurun_out/${TAG}_bench_default.json 2> gpurun_out/${TAG}_bench_default.err || { echo "bench rc=$?"; tail -20 gpurun_out/${TAG}_bench_default.err; exit 1; }
python -c "import json; r=json.load(open('gpurun_out/${TAG}_bench_default.json')); c=r['cpu_baseline']; print('default', r['value'], r['ms_per_step'], r['roofline']['kernel'], r['roofline']['frac'], 'cpu', c.get('value'), c.get('threads_used'), c.get('step_s'))"
echo done
