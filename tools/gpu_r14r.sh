# the direct-load 1x1 GEMM: its tests, per-call A/B against the LDS kernel
# (standalone builds), the probe trace, the bench
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_conv1x1.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/r14r_tests.txt 2>&1 || { echo "tests rc=$?"; tail -30 gpurun_out/r14r_tests.txt; exit 1; }
tail -1 gpurun_out/r14r_tests.txt
timeout -k 10 300 python -u tools/c1_probe.py --libs c1_base,c1_old,c1_base,c1_old > gpurun_out/r14r_probe.txt 2>&1 || { echo "probe rc=$?"; tail -20 gpurun_out/r14r_probe.txt; exit 1; }
grep -v "^{\|amdgpu" gpurun_out/r14r_probe.txt
timeout -k 10 400 python bench.py --steps 30 --warmup 5 --no-cpu-baseline --mmd-sweep 0 --ref-schedule-steps 0 > gpurun_out/r14r_bench.json 2> gpurun_out/r14r_bench.err || { echo "bench rc=$?"; tail -20 gpurun_out/r14r_bench.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/r14r_bench.json'));print('bench',d['value'],d['ms_per_step'])"
