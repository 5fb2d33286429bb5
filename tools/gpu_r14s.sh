# 1x1 weight-gradient chunk width / slicing variants (standalone builds) + tests
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_conv1x1.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/r14s_tests.txt 2>&1 || { echo "tests rc=$?"; tail -30 gpurun_out/r14s_tests.txt; exit 1; }
tail -1 gpurun_out/r14s_tests.txt
timeout -k 10 300 python -u tools/c1_probe.py --libs c1_base,c1_w64,c1_w64m4,c1_w64m16,c1_m16 > gpurun_out/r14s_probe.txt 2>&1 || { echo "probe rc=$?"; tail -20 gpurun_out/r14s_probe.txt; exit 1; }
grep -v "^{\|amdgpu" gpurun_out/r14s_probe.txt | grep "dw\|case\|sum"
