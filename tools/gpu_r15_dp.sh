# DP checks + world-1 RCCL vs group-less A/B: bash tools/gpu_r15_dp.sh TAG
set -o pipefail
TAG=${1:-r15dp}
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_dist.py tests/test_gpu_model.py -k "dist or rccl or two_ranks or tower or bit_identical or late" > gpurun_out/${TAG}_tests.txt 2>&1 || { echo "tests rc=$?"; tail -40 gpurun_out/${TAG}_tests.txt; exit 1; }
tail -2 gpurun_out/${TAG}_tests.txt
B="--steps 30 --warmup 6 --no-cpu-baseline --mmd-sweep 0 --ref-schedule-steps 0 --instrument-cycles 0"
for r in 1 2 3; do
  SMMD_DP_FORCE=1 timeout -k 10 400 python bench.py $B > gpurun_out/${TAG}_rccl1_$r.json 2> gpurun_out/${TAG}_rccl1_$r.err || { echo "bench rccl rc=$?"; tail -20 gpurun_out/${TAG}_rccl1_$r.err; exit 1; }
  python -c "import json; r=json.load(open('gpurun_out/${TAG}_rccl1_$r.json')); print('rccl world1 run $r', r['value'], r['ms_per_step'], r['config'].get('parallelism'))"
  timeout -k 10 400 python bench.py $B > gpurun_out/${TAG}_nogroup_$r.json 2> gpurun_out/${TAG}_nogroup_$r.err || { echo "bench nogroup rc=$?"; exit 1; }
  python -c "import json; r=json.load(open('gpurun_out/${TAG}_nogroup_$r.json')); print('group-less run $r', r['value'], r['ms_per_step'])"
done
echo done
