# Targeted GPU tests (pytest -k expression) then optional extra command:
# bash tools/gpu_quick.sh TAG 'k-expr' [files...]
set -o pipefail
TAG=${1:-quick}
K=${2:-smmd_loss}
shift 2
FILES=${@:-tests}
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest $FILES -m gpu -x -q --timeout 300 --timeout-method thread -k "$K" > gpurun_out/${TAG}_tests.txt 2>&1 || { echo "tests rc=$?"; tail -40 gpurun_out/${TAG}_tests.txt; exit 1; }
tail -2 gpurun_out/${TAG}_tests.txt
