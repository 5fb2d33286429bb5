# Interleaved A/B (off, on, off, on) of one library build under an env toggle
# on the forward Winograd kernels alone:
#   bash tools/gpu_ab_env.sh TAG VAR [only]     (VAR=0 is "off", unset is "on")
set -o pipefail
TAG=${1:-abe}
VAR=${2:-SMMD_WINO8}
ONLY=${3:-}
mkdir -p gpurun_out
for arm in off on off on; do
  if [ $arm = off ]; then export $VAR=0; else unset $VAR; fi
  timeout -k 10 120 python -u tools/wino_pmc.py --iters 50 ${ONLY:+--only $ONLY} > gpurun_out/${TAG}_${arm}.txt 2>&1 || { echo "$arm rc=$?"; tail -5 gpurun_out/${TAG}_${arm}.txt; exit 1; }
  echo "== $arm"; tail -1 gpurun_out/${TAG}_${arm}.txt | python -c "import sys,json; d=json.loads(sys.stdin.read()); [print(k, v['us'], v['mfma_frac'], v.get('clock_ghz')) for k, v in d.items() if isinstance(v, dict)]"
done
unset $VAR
