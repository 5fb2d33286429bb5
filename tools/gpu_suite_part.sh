# A part of the GPU suite in the suite's order: bash tools/gpu_suite_part.sh TAG FILES...
set -o pipefail
TAG=$1; shift
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest "$@" -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/${TAG}.txt 2>&1; rc=$?
tail -3 gpurun_out/${TAG}.txt
[ $rc -eq 0 ] || { grep -E "FAILED|Error|^E " gpurun_out/${TAG}.txt | head -20; exit 1; }
echo done
