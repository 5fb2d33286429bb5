# Elementwise sources of the current tree (torch profiler, D and G steps).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u tools/op_sources.py --top 80 > gpurun_out/r14o_opsrc.txt 2>&1 || { echo "opsrc rc=$?"; tail -20 gpurun_out/r14o_opsrc.txt; exit 1; }
grep "==" gpurun_out/r14o_opsrc.txt
