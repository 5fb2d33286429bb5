set -o pipefail
mkdir -p gpurun_out
timeout -k 5 120 ./tools/hip/mmd_abi_bench > gpurun_out/r04c_abi.txt || exit 1
cat gpurun_out/r04c_abi.txt
timeout -k 10 1200 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r04c_tests.txt 2>&1 || { echo "tests rc=$?"; tail -40 gpurun_out/r04c_tests.txt; exit 1; }
tail -1 gpurun_out/r04c_tests.txt
