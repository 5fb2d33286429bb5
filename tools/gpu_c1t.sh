# 1x1 input gradient straight from W (smmd_conv1x1_t, ABI 16): tests + kernel-time and bench A/B
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_conv1x1.py tests/test_gpu_model.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/c1t_tests.txt 2>&1 || { echo "tests rc=$?"; tail -30 gpurun_out/c1t_tests.txt; exit 1; }
tail -1 gpurun_out/c1t_tests.txt
for v in 1 0; do
  SMMD_C1_DX_T=$v timeout -s KILL 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/c1tt_$v -o run -- python tools/step_cycle.py --cycles 2 > gpurun_out/c1tt_$v.log 2>&1 || { echo "trace rc=$?"; exit 1; }
done
python - <<'PY'
import csv, glob
for v in ('1', '0'):
    f = glob.glob('gpurun_out/c1tt_%s/**/run_kernel_stats.csv' % v, recursive=True)[0]
    rows = list(csv.DictReader(open(f)))
    tot = sum(float(r['TotalDurationNs']) for r in rows)
    c1 = sum(float(r['TotalDurationNs']) for r in rows if 'c1_gemm' in r['Name'])
    cp = sum(float(r['TotalDurationNs']) for r in rows if 'elementwise' in r['Name'] and ('copy' in r['Name'].lower() or 'direct_copy' in r['Name']))
    print('SMMD_C1_DX_T=%s kernel total %.3f ms  c1_gemm %.3f ms  torch copies %.3f ms (12 steps)' % (v, tot / 1e6, c1 / 1e6, cp / 1e6))
PY
for r in 1 2; do
  for v in 1 0; do
    SMMD_C1_DX_T=$v timeout -k 10 400 python bench.py --steps 40 --warmup 5 --no-cpu-baseline --mmd-sweep 0 --ref-schedule-steps 0 > gpurun_out/c1t_${v}_${r}.json 2> gpurun_out/c1t_${v}_${r}.err || { echo "bench rc=$?"; tail -20 gpurun_out/c1t_${v}_${r}.err; exit 1; }
    python -c "import json;d=json.load(open('gpurun_out/c1t_${v}_${r}.json'));print('SMMD_C1_DX_T=$v run $r',d['value'],d['ms_per_step'])"
  done
done
echo done
