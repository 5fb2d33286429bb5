# Interleaved A/B (base, new, base, new) of two library builds on the forward
# Winograd kernels alone: bash tools/gpu_ab_wino.sh TAG BASE_SO [only]
set -o pipefail
TAG=${1:-abw}
BASE=${2:-tools/hip/ab_base.so}
ONLY=${3:-}
NEW=scaled-mmd-gan_amd/lib/libsmmd_hip.so
mkdir -p gpurun_out
for arm in base new base new; do
  L=$BASE; [ $arm = new ] && L=$NEW
  timeout -k 10 120 python -u tools/wino_pmc.py --lib $L --iters 50 ${ONLY:+--only $ONLY} > gpurun_out/${TAG}_${arm}.txt 2>&1 || { echo "$arm rc=$?"; tail -5 gpurun_out/${TAG}_${arm}.txt; exit 1; }
  echo "== $arm"; tail -1 gpurun_out/${TAG}_${arm}.txt | python -c "import sys,json; d=json.loads(sys.stdin.read()); [print(k, v['us'], v['mfma_frac'], v.get('clock_ghz')) for k, v in d.items() if isinstance(v, dict)]"
done
