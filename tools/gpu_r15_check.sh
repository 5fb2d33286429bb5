# round-6 checks: the DP / graph / determinism tests, then interleaved bench A/Bs
# bash tools/gpu_r15_check.sh TAG
set -o pipefail
TAG=${1:-r15}
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_dist.py tests/test_gpu_model.py -k "dist or rccl or graphs or bit_identical or two_ranks or tower" > gpurun_out/${TAG}_tests.txt 2>&1 || { echo "tests rc=$?"; tail -40 gpurun_out/${TAG}_tests.txt; exit 1; }
tail -3 gpurun_out/${TAG}_tests.txt
B="--steps 30 --warmup 6 --no-cpu-baseline --mmd-sweep 0 --ref-schedule-steps 0 --instrument-cycles 0"
for r in 1 2; do
  for v in 0 1; do
    timeout -k 10 400 python bench.py $B --graphs $v > gpurun_out/${TAG}_graphs${v}_$r.json 2> gpurun_out/${TAG}_graphs${v}_$r.err || { echo "bench graphs=$v rc=$?"; tail -20 gpurun_out/${TAG}_graphs${v}_$r.err; exit 1; }
    python -c "import json; r=json.load(open('gpurun_out/${TAG}_graphs${v}_$r.json')); print('graphs=$v run $r', r['value'], r['ms_per_step'])"
  done
done
for r in 1 2; do
  for v in 0 1; do
    SMMD_DP_FORCE=1 SMMD_GLOBAL_FUSED_LOSS=$v timeout -k 10 400 python bench.py $B > gpurun_out/${TAG}_rccl1_fused${v}_$r.json 2> gpurun_out/${TAG}_rccl1_fused${v}_$r.err || { echo "bench rccl fused=$v rc=$?"; tail -20 gpurun_out/${TAG}_rccl1_fused${v}_$r.err; exit 1; }
    python -c "import json; r=json.load(open('gpurun_out/${TAG}_rccl1_fused${v}_$r.json')); print('rccl world1 fused=$v run $r', r['value'], r['ms_per_step'], r['config'].get('parallelism'))"
  done
  timeout -k 10 400 python bench.py $B > gpurun_out/${TAG}_nogroup_$r.json 2> gpurun_out/${TAG}_nogroup_$r.err || { echo "bench nogroup rc=$?"; exit 1; }
  python -c "import json; r=json.load(open('gpurun_out/${TAG}_nogroup_$r.json')); print('group-less run $r', r['value'], r['ms_per_step'])"
done
echo done
