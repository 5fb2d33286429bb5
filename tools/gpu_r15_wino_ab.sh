# V-stage layout A/B of the 8-wave 3x3 kernel (interleaved): bash tools/gpu_r15_wino_ab.sh TAG
set -o pipefail
TAG=${1:-r15w}
mkdir -p gpurun_out
for r in 1 2; do
  for L in tools/hip/v_vpair0.so scaled-mmd-gan_amd/lib/libsmmd_hip.so tools/hip/v_novs0.so tools/hip/v_novs.so; do
    n=$(basename $L .so)
    timeout -k 10 120 python -u tools/wino_pmc.py --lib $L --iters 50 --only 3x3 > gpurun_out/${TAG}_${n}_$r.txt 2>&1 || { echo "$n rc=$?"; tail -5 gpurun_out/${TAG}_${n}_$r.txt; exit 1; }
    echo "== $n run $r"; tail -1 gpurun_out/${TAG}_${n}_$r.txt | python -c "import sys,json; d=json.loads(sys.stdin.read()); [print(k, v['us'], v['mfma_frac']) for k, v in d.items() if isinstance(v, dict)]"
  done
done
