# One round-3 GPU pass: the -m gpu suite, the 2-rank launch through
# `bench.py --gpus 2` itself (gloo, both ranks on the one GPU), and the
# default bench.  bash tools/gpu_round.sh TAG
set -o pipefail
TAG=${1:-r07}
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/${TAG}_gpu_tests.txt 2>&1 || { echo "tests rc=$?"; tail -40 gpurun_out/${TAG}_gpu_tests.txt; exit 1; }
tail -2 gpurun_out/${TAG}_gpu_tests.txt
SMMD_DIST_BACKEND=gloo SMMD_SAME_DEVICE=1 timeout -k 10 300 python bench.py --gpus 2 --steps 12 --warmup 6 --no-cpu-baseline --mmd-sweep 2 --ref-schedule-steps 0 > gpurun_out/${TAG}_bench2.json 2> gpurun_out/${TAG}_bench2.err || { echo "bench2 rc=$?"; tail -30 gpurun_out/${TAG}_bench2.err; exit 1; }
python -c "import json; r=json.loads([l for l in open('gpurun_out/${TAG}_bench2.json') if l.startswith('{')][-1]); print('2 ranks', r['value'], r['n_gpus'], r['config']['parallelism'], r['ms_per_step'])"
timeout -k 10 900 python bench.py > gpurun_out/${TAG}_bench_default.json 2> gpurun_out/${TAG}_bench_default.err || { echo "bench rc=$?"; tail -20 gpurun_out/${TAG}_bench_default.err; exit 1; }
python -c "import json; r=json.load(open('gpurun_out/${TAG}_bench_default.json')); c=r['cpu_baseline']; print('default', r['value'], r['ms_per_step'], r['roofline']['kernel'], r['roofline']['frac'], 'cpu', c.get('value'), c.get('threads_used'), c.get('step_s'))"
echo done
