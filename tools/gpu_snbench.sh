# Kernel times of the SN refresh variants (tools/sn_bench.py), one rocprofv3
# kernel trace per mode: bash tools/gpu_snbench.sh TAG
set -o pipefail
TAG=${1:-snb}
mkdir -p gpurun_out
export TMPDIR=/tmp
for M in ${MODES:-0: 1: 1:1 1:2 1:3 1:4 1:8 1:12}; do
  D=gpurun_out/${TAG}_${M/:/_}
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $D -o run -- python tools/sn_bench.py 40 $M > $D.log 2>&1 || { echo "mode $M rc=$?"; tail -5 $D.log; exit 1; }
  echo "== mode $M"; grep -h "P23" $D.log
  python - $D <<'PY'
import csv, glob, sys
f = glob.glob(sys.argv[1] + '/**/*kernel_stats.csv', recursive=True)[0]
for r in csv.DictReader(open(f)):
    if 'sn_' in r['Name']:
        print('  %-40s n %5s avg %8.2f us' % (r['Name'][:40], r['Calls'], float(r['AverageNs']) / 1e3))
PY
done
