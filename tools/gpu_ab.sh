# A/B of bench variants on one box: bash tools/gpu_ab.sh TAG "args A" "args B" ...
set -o pipefail
TAG=$1; shift
mkdir -p gpurun_out
export TMPDIR=/tmp
i=0
for a in "$@"; do
  i=$((i+1))
  echo "[ab] variant $i: $a"
  timeout -k 10 600 python bench.py --no-cpu-baseline $a > gpurun_out/${TAG}_v$i.json 2> gpurun_out/${TAG}_v$i.err || { echo "variant $i rc=$?"; tail -20 gpurun_out/${TAG}_v$i.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/${TAG}_v$i.json'));print(d['value'], d['ms_per_step'], d['config'].get('memory_format'), d['config'].get('miopen_winograd'))"
done
