# A/B of a bench.py flag, interleaved: bash tools/gpu_ab_flag.sh TAG "--flag A" "--flag B"
set -o pipefail
TAG=${1:-abflag}
A=${2:-}
B=${3:-}
mkdir -p gpurun_out
export TMPDIR=/tmp
for r in 1 2; do
  for v in a b; do
    if [ $v = a ]; then F="$A"; else F="$B"; fi
    timeout -k 10 600 python bench.py --steps 30 --warmup 6 --no-cpu-baseline --mmd-sweep 0 --ref-schedule-steps 0 $F > gpurun_out/${TAG}_${v}_${r}.json 2> gpurun_out/${TAG}_${v}_${r}.err || { echo "bench $v rc=$?"; tail -20 gpurun_out/${TAG}_${v}_${r}.err; exit 1; }
    python -c "import json; r=json.load(open('gpurun_out/${TAG}_${v}_${r}.json')); print('[$F] run $r', r['value'], r['ms_per_step'], r['step_ms_by_kind'])"
  done
done
echo done
