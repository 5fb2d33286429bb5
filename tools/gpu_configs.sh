# bench.py on BASELINE configs[1] (cifar10) and [2] (celebA 64x64): bash tools/gpu_configs.sh TAG
set -o pipefail
TAG=${1:-cfg}
mkdir -p gpurun_out
for C in cifar10 celebA64; do
  echo "[cfg] $C"
  timeout -k 10 500 python bench.py --config $C --steps 30 --warmup 6 --no-cpu-baseline --mmd-sweep 0 > gpurun_out/${TAG}_$C.json 2> gpurun_out/${TAG}_$C.err || { echo "$C rc=$?"; tail -20 gpurun_out/${TAG}_$C.err; exit 1; }
  python -c "import json; r=json.load(open('gpurun_out/${TAG}_$C.json')); print('$C', r['value'], r['ms_per_step'], r['step_ms_by_kind'], r['schedule_reference']['value'])"
done
echo done
