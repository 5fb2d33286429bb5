# Interleaved A/B of several library builds on the Winograd kernels (one box):
# bash tools/gpu_abn.sh TAG ONLY ROUNDS LIB1 LIB2 ...   (ONLY: 3x3|s2|s2t|wgrad|'')
set -o pipefail
TAG=$1; ONLY=$2; ROUNDS=$3; shift 3
mkdir -p gpurun_out
for r in $(seq 1 $ROUNDS); do
  i=0
  for L in "$@"; do
    i=$((i+1))
    timeout -k 10 120 python -u tools/wino_pmc.py --lib $L --iters 50 ${ONLY:+--only $ONLY} > gpurun_out/${TAG}_${r}_${i}.txt 2>&1 || { echo "$L rc=$?"; tail -5 gpurun_out/${TAG}_${r}_${i}.txt; exit 1; }
    echo "== round $r $(basename $L)"; tail -1 gpurun_out/${TAG}_${r}_${i}.txt | python -c "import sys,json; d=json.loads(sys.stdin.read()); print(' '.join('%s:%s/%s' % (k, v['us'], v['mfma_frac']) for k, v in d.items() if isinstance(v, dict)))"
  done
done
