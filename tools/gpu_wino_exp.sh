# Timing of experimental library builds (tools/hip/exp*.so) on the 3x3
# forward kernel: bash tools/gpu_wino_exp.sh TAG so...
set -o pipefail
TAG=$1; shift
mkdir -p gpurun_out
for L in scaled-mmd-gan_amd/lib/libsmmd_hip.so "$@"; do
  timeout -k 10 120 python -u tools/wino_pmc.py --lib $L --iters 50 --only 3x3 > gpurun_out/${TAG}_$(basename $L).txt 2>&1 || { echo "$L rc=$?"; tail -5 gpurun_out/${TAG}_$(basename $L).txt; exit 1; }
  echo "== $L"; tail -1 gpurun_out/${TAG}_$(basename $L).txt | python -c "import sys,json; d=json.loads(sys.stdin.read()); [print(k, v['us'], v['mfma_frac'], v.get('clock_ghz')) for k, v in d.items() if isinstance(v, dict)]"
done
