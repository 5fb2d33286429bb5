set -o pipefail
for cfg in "1024 32" "512 32" "2048 32" "512 64"; do
  set -- $cfg
  echo "== blocks=$1 mincpw=$2"
  SMMD_TILE_BLOCKS=$1 SMMD_TILE_MINCPW=$2 timeout -k 5 120 ./tools/hip/mmd_abi_bench | tr '\n' ' ' || exit 1
  echo
done
echo "== row sweep"
SMMD_MMD_TILE=0 timeout -k 5 120 ./tools/hip/mmd_abi_bench | tr '\n' ' ' || exit 1
echo
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py -x -q -k "mmd2" --timeout 300 --timeout-method thread > gpurun_out/mmdt3_tests.txt 2>&1 || { echo "tests rc=$?"; tail -40 gpurun_out/mmdt3_tests.txt; exit 1; }
tail -1 gpurun_out/mmdt3_tests.txt
