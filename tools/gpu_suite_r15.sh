# The GPU suite, smoke() and the host probe on the final tree: bash tools/gpu_suite_r15.sh TAG
set -o pipefail
TAG=${1:-suite15}
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > gpurun_out/${TAG}_gpu_tests.txt 2>&1; rc=$?
tail -3 gpurun_out/${TAG}_gpu_tests.txt
[ $rc -eq 0 ] || { grep -E "FAILED|Error" gpurun_out/${TAG}_gpu_tests.txt | head -20; exit 1; }
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${TAG}_smoke.txt 2>&1 || { echo "smoke rc=$?"; tail -20 gpurun_out/${TAG}_smoke.txt; exit 1; }
cat gpurun_out/${TAG}_smoke.txt | tail -1
timeout -k 10 300 python tools/host_probe.py > gpurun_out/${TAG}_host_probe.txt 2>&1 || { echo "host probe rc=$?"; tail -20 gpurun_out/${TAG}_host_probe.txt; exit 1; }
tail -5 gpurun_out/${TAG}_host_probe.txt
echo done
