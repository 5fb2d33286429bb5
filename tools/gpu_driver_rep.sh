# the driver's bench command three times back to back (run-to-run spread)
set -o pipefail
mkdir -p gpurun_out
for i in 1 2 3; do
  timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/drv_$i.json 2> gpurun_out/drv_$i.err || { echo "rc=$?"; tail -5 gpurun_out/drv_$i.err; exit 1; }
  python -c "import json; r=json.load(open('gpurun_out/drv_$i.json')); print('driver', r['value'], r['ms_per_step'], r['d_steps'], r['g_steps'], r.get('cycle_value'))"
done
