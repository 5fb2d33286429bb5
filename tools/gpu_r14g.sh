# Where the step's elementwise kernels come from (autograd node attribution),
# the 1x1 shortcut convs on MIOpen vs GEMM forms, and a kernel trace of two
# whole 5D+1G cycles of the current tree.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u tools/op_sources.py --top 60 > gpurun_out/r14g_opsrc.txt 2>&1 || { echo "opsrc rc=$?"; tail -20 gpurun_out/r14g_opsrc.txt; exit 1; }
grep "==" gpurun_out/r14g_opsrc.txt
timeout -k 10 300 python -u tools/conv1x1_bench.py > gpurun_out/r14g_1x1.txt 2>&1 || { echo "1x1 rc=$?"; tail -20 gpurun_out/r14g_1x1.txt; exit 1; }
cat gpurun_out/r14g_1x1.txt | grep "{"
timeout -s KILL 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r14g_trace -o run -- python tools/step_cycle.py --cycles 2 > gpurun_out/r14g_trace.log 2>&1 || { echo "trace rc=$?"; exit 1; }
echo done
