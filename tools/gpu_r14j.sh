# 1x1 shortcut convs: library vs MIOpen per call, and a kernel trace of two
# whole 5D+1G cycles on the current tree.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u tools/conv1x1_bench.py > gpurun_out/r14j_1x1.txt 2>&1 || { echo "1x1 rc=$?"; tail -20 gpurun_out/r14j_1x1.txt; exit 1; }
grep "{" gpurun_out/r14j_1x1.txt
timeout -s KILL 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r14j_trace -o run -- python tools/step_cycle.py --cycles 2 > gpurun_out/r14j_trace.log 2>&1 || { echo "trace rc=$?"; exit 1; }
echo done
