# Library 1x1 convs (register-staged, reads-first, per-kernel slicing): the
# whole gpu suite, an interleaved A/B of SMMD_CONV1X1 on the bench, the
# 1x1 probe and a kernel trace of two whole 5D+1G cycles.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/r14n_tests.txt 2>&1 || { echo "tests rc=$?"; tail -30 gpurun_out/r14n_tests.txt; exit 1; }
tail -1 gpurun_out/r14n_tests.txt
for r in 1 2; do
  for v in 0 1; do
    SMMD_CONV1X1=$v timeout -k 10 400 python bench.py --steps 30 --warmup 5 --no-cpu-baseline --mmd-sweep 0 --ref-schedule-steps 0 > gpurun_out/r14n_ab_${v}_${r}.json 2> gpurun_out/r14n_ab_${v}_${r}.err || { echo "bench rc=$?"; tail -20 gpurun_out/r14n_ab_${v}_${r}.err; exit 1; }
    python -c "import json;d=json.load(open('gpurun_out/r14n_ab_${v}_${r}.json'));print('SMMD_CONV1X1=$v run $r',d['value'],d['ms_per_step'],d['step_ms_by_kind'])"
  done
done
timeout -k 10 300 python -u tools/c1_probe.py --libs lib > gpurun_out/r14n_probe.txt 2>&1 || { echo "probe rc=$?"; exit 1; }
timeout -s KILL 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r14n_trace -o run -- python tools/step_cycle.py --cycles 2 > gpurun_out/r14n_trace.log 2>&1 || { echo "trace rc=$?"; exit 1; }
echo done
