# Round-5 final tree: the whole GPU suite and smoke().
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/r14_final_tests.txt 2>&1 || { echo "tests rc=$?"; tail -30 gpurun_out/r14_final_tests.txt; exit 1; }
tail -1 gpurun_out/r14_final_tests.txt
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r14_final_smoke.txt 2>&1 || { echo "smoke rc=$?"; tail -20 gpurun_out/r14_final_smoke.txt; exit 1; }
tail -2 gpurun_out/r14_final_smoke.txt
