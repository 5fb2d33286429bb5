# V point-block padding A/B of the 8-wave 3x3 kernel (interleaved): bash tools/gpu_r15_vpad_ab.sh TAG
set -o pipefail
TAG=${1:-r15vp}
mkdir -p gpurun_out
for r in 1 2 3; do
  for L in tools/hip/v_vpad0.so scaled-mmd-gan_amd/lib/libsmmd_hip.so; do
    n=$(basename $L .so)
    timeout -k 10 120 python -u tools/wino_pmc.py --lib $L --iters 50 --only 3x3 > gpurun_out/${TAG}_${n}_$r.txt 2>&1 || { echo "$n rc=$?"; tail -5 gpurun_out/${TAG}_${n}_$r.txt; exit 1; }
    echo "== $n run $r"; tail -1 gpurun_out/${TAG}_${n}_$r.txt | python -c "import sys,json; d=json.loads(sys.stdin.read()); [print(k, v['us'], v['mfma_frac']) for k, v in d.items() if isinstance(v, dict)]"
  done
done
timeout -k 10 300 python -u -m pytest tests/test_gpu_wino.py -x -q --timeout 200 --timeout-method thread > gpurun_out/${TAG}_tests.txt 2>&1 || { echo "tests rc=$?"; tail -20 gpurun_out/${TAG}_tests.txt; exit 1; }
tail -1 gpurun_out/${TAG}_tests.txt
