# Interleaved timing of several library builds on the forward Winograd
# kernels (two rounds): bash tools/gpu_ab_libs.sh TAG ONLY LIB1 LIB2 ...
set -o pipefail
TAG=$1; ONLY=$2; shift 2
mkdir -p gpurun_out
for r in 1 2; do
  for L in "$@"; do
    n=$(basename $L .so)
    timeout -k 10 120 python -u tools/wino_pmc.py --lib $L --iters 50 ${ONLY:+--only $ONLY} > gpurun_out/${TAG}_${n}_$r.txt 2>&1 || { echo "$n rc=$?"; tail -5 gpurun_out/${TAG}_${n}_$r.txt; exit 1; }
    echo "== $n"; tail -1 gpurun_out/${TAG}_${n}_$r.txt | python -c "import sys,json; d=json.loads(sys.stdin.read()); print(' '.join(f\"{k}:{v['us']}/{v['mfma_frac']}\" for k, v in d.items() if isinstance(v, dict)))"
  done
done
