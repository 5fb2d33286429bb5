# kernel-time A/B of SMMD_GY_ACC over two step cycles (rocprofv3 kernel trace)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
for v in 1 0; do
  SMMD_GY_ACC=$v timeout -s KILL 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/gyt_$v -o run -- python tools/step_cycle.py --cycles 2 > gpurun_out/gyt_$v.log 2>&1 || { echo "trace rc=$?"; exit 1; }
done
python - <<'PY'
import csv, glob
for v in ('1', '0'):
    f = glob.glob('gpurun_out/gyt_%s/**/run_kernel_stats.csv' % v, recursive=True)[0]
    rows = list(csv.DictReader(open(f)))
    tot = sum(float(r['TotalDurationNs']) for r in rows)
    s2 = sum(float(r['TotalDurationNs']) for r in rows if 's2_conv_kernel' in r['Name'] or 's2_reduce' in r['Name'])
    add = sum(float(r['TotalDurationNs']) for r in rows if 'CUDAFunctor_add' in r['Name'])
    print('SMMD_GY_ACC=%s total %.3f ms  s2 conv+reduce %.3f ms  torch add %.3f ms' % (v, tot / 1e6, s2 / 1e6, add / 1e6))
PY
