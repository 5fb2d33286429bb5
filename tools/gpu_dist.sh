# N > 1 rehearsal on ONE GPU box: bash tools/gpu_dist.sh TAG
#  1. the 2-rank global-mode test (gloo, both ranks on cuda:0) + the model tests
#  2. bench.py under torch.distributed.run with 2 ranks sharing the GPU (gloo)
set -o pipefail
TAG=${1:-dist}
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_dist.py tests/test_gpu_model.py -x -v --timeout 240 --timeout-method thread -m gpu > gpurun_out/${TAG}_tests.log 2>&1 || { echo "tests rc=$?"; tail -30 gpurun_out/${TAG}_tests.log; exit 1; }
tail -3 gpurun_out/${TAG}_tests.log
SMMD_DIST_BACKEND=gloo SMMD_SAME_DEVICE=1 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 2 --steps 6 --warmup 6 --no-cpu-baseline --mmd-sweep 2 --ref-schedule-steps 0 > gpurun_out/${TAG}_bench2.json 2> gpurun_out/${TAG}_bench2.err || { echo "bench2 rc=$?"; tail -30 gpurun_out/${TAG}_bench2.err; exit 1; }
head -c 400 gpurun_out/${TAG}_bench2.json
echo
echo done
