# SN refresh / grad-stats changes: the whole gpu suite, the SN A/B against the
# round-start build, a kernel trace of sn_bench, the driver's bench command.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/r14f_tests.txt 2>&1 || { echo "tests rc=$?"; tail -30 gpurun_out/r14f_tests.txt; exit 1; }
tail -1 gpurun_out/r14f_tests.txt
for r in 1 2; do
  for L in tools/hip/v_r14base.so scaled-mmd-gan_amd/lib/libsmmd_hip.so; do
    SMMD_HIP_LIB=$L timeout -k 10 120 python -u tools/sn_bench.py --iters 200 > gpurun_out/r14f_sn_${r}_$(basename $L .so).txt 2>&1 || { echo "$L rc=$?"; exit 1; }
    echo "== round $r $(basename $L)"; tail -1 gpurun_out/r14f_sn_${r}_$(basename $L .so).txt | python -c "import sys,json; d=json.loads(sys.stdin.read()); print(' '.join('%s:%s' % (k, v['avg_us']) for k, v in d.items() if isinstance(v, dict)))"
  done
done
timeout -k 10 180 rocprofv3 --kernel-trace --stats -d gpurun_out/r14f_prof -o sn -- python3 tools/sn_bench.py --iters 100 > gpurun_out/r14f_prof.log 2>&1 || { echo "prof rc=$?"; exit 1; }
timeout -k 10 400 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --mmd-sweep 0 --ref-schedule-steps 0 > gpurun_out/r14f_bench.json 2> gpurun_out/r14f_bench.err || { echo "bench rc=$?"; tail -20 gpurun_out/r14f_bench.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/r14f_bench.json'));print('bench',d['value'],d['ms_per_step'],d['step_ms_by_kind'],d['roofline']['kernel'],d['roofline']['frac']);h=d['roofline_hot_path'];print({k:(h[k].get('avg_ms'),h[k].get('hbm_frac')) for k in ('smmd_sn_power_iter','smmd_sn_grad_stats') if k in h})"
echo done
