# Multi-rank path on the one-GPU box: the 2-rank GPU test (gloo, both ranks on
# cuda:0, the real kernels) and bench.py --gpus 2 through its own launcher.
# bash tools/gpu_dist.sh TAG
set -o pipefail
TAG=${1:-dist}
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_dist.py -m gpu -x -v --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/${TAG}_tests.txt 2>&1 || { echo "tests rc=$?"; tail -30 gpurun_out/${TAG}_tests.txt; exit 1; }
tail -3 gpurun_out/${TAG}_tests.txt
SMMD_DIST_BACKEND=gloo SMMD_SAME_DEVICE=1 timeout -k 10 500 python bench.py --gpus 2 --steps 12 --warmup 6 --no-cpu-baseline --mmd-sweep 0 --ref-schedule-steps 0 --instrument-cycles 1 > gpurun_out/${TAG}_bench2.json 2> gpurun_out/${TAG}_bench2.err || { echo "bench rc=$?"; tail -20 gpurun_out/${TAG}_bench2.err; exit 1; }
grep "^{" gpurun_out/${TAG}_bench2.json | python -c "import json,sys;d=json.loads(sys.stdin.read());print(d['value'],d['n_gpus'],d['config']['parallelism'],d['ms_per_step'],{k:v for k,v in d['hip_kernels'].items() if 'sn' in k})"
