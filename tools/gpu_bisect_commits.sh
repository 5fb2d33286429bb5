# the global-mode 2-rank test in older trees (bisect_wt/<commit>, built in place)
set -o pipefail
mkdir -p gpurun_out
for c in "$@"; do
  (cd bisect_wt/$c && timeout -k 10 200 python -u -m pytest tests/test_gpu_dist.py -m gpu -x -q -k global_mode --timeout 150 --timeout-method thread -p no:cacheprovider > ../../gpurun_out/bisect_c_$c.txt 2>&1)
  echo "$c rc=$? $(tail -1 gpurun_out/bisect_c_$c.txt)"
done
