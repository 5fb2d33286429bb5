# test_global_mode_two_ranks_equal_one_process under env toggles: bash tools/gpu_bisect_dist.sh
set -o pipefail
mkdir -p gpurun_out
for v in "$@"; do
  env $v timeout -k 10 200 python -u -m pytest tests/test_gpu_dist.py -m gpu -x -q -k global_mode --timeout 150 --timeout-method thread -p no:cacheprovider > gpurun_out/bisect_$v.txt 2>&1
  echo "$v rc=$? $(tail -1 gpurun_out/bisect_$v.txt)"
done
