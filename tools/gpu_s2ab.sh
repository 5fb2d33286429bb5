# Interleaved A/B of a stride-2 variant build (tools/hip/v_NAME.so) against the
# stamped library on the forward and transposed stride-2 kernels:
#   bash tools/gpu_s2ab.sh TAG NAME
set -o pipefail
TAG=${1:-s2ab}
V=tools/hip/v_${2}.so
mkdir -p gpurun_out
for only in s2 s2t; do
  for arm in lib var lib var; do
    L=scaled-mmd-gan_amd/lib/libsmmd_hip.so; [ $arm = var ] && L=$V
    timeout -k 10 120 python -u tools/wino_pmc.py --lib $L --iters 50 --only $only > gpurun_out/${TAG}_${only}_${arm}.txt 2>&1 || { echo "$arm rc=$?"; tail -5 gpurun_out/${TAG}_${only}_${arm}.txt; exit 1; }
    echo "== $only $arm"; tail -1 gpurun_out/${TAG}_${only}_${arm}.txt | python -c "import sys,json; d=json.loads(sys.stdin.read()); print(' '.join('%s %s/%s' % (k, v['us'], v['mfma_frac']) for k, v in d.items() if isinstance(v, dict)))"
  done
done
