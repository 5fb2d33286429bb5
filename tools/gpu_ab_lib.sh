# A/B of two library builds on the Winograd bench, interleaved (base, new,
# base, new) on one box: bash tools/gpu_ab_lib.sh TAG BASE_SO [bench script]
set -o pipefail
TAG=${1:-ab}
BASE=${2:-tools/hip/ab_base.so}
BENCH=${3:-tools/wino_bench.py}
NEW=scaled-mmd-gan_amd/lib/libsmmd_hip.so
mkdir -p gpurun_out
for arm in base new base new; do
  L=$BASE; [ $arm = new ] && L=$NEW
  timeout -k 10 300 python -u $BENCH --lib $L --iters 20 > gpurun_out/${TAG}_${arm}.txt 2>&1 || { echo "$arm rc=$?"; tail -5 gpurun_out/${TAG}_${arm}.txt; exit 1; }
  echo "== $arm"; grep '^{' gpurun_out/${TAG}_${arm}.txt | python -c "import sys,json; [print(r['shape'], 'wino_us', round(r['wino_us'],1), 'frac', round(r['executed_tflops_wino']/157.3,3)) for r in map(json.loads, sys.stdin)]"
done
