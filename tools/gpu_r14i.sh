# Library UpsampleConv fold + host BN counter: the fold / relupool / model gpu
# tests, then the driver's bench command and the elementwise sources again.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/r14i_tests.txt 2>&1 || { echo "tests rc=$?"; tail -30 gpurun_out/r14i_tests.txt; exit 1; }
tail -1 gpurun_out/r14i_tests.txt
timeout -k 10 400 python bench.py --steps 30 --warmup 5 --no-cpu-baseline --mmd-sweep 0 --ref-schedule-steps 0 > gpurun_out/r14i_bench.json 2> gpurun_out/r14i_bench.err || { echo "bench rc=$?"; tail -20 gpurun_out/r14i_bench.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/r14i_bench.json'));print('bench',d['value'],d['ms_per_step'],d['step_ms_by_kind'],d['roofline']['kernel'],d['roofline']['frac'])"
timeout -k 10 300 python -u tools/op_sources.py --top 40 > gpurun_out/r14i_opsrc.txt 2>&1 || { echo "opsrc rc=$?"; exit 1; }
grep "==" gpurun_out/r14i_opsrc.txt
echo done
