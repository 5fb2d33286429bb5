# The driver's bench command with the Winograd weight gradient on / off (GPU box)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
for v in 1 0 1; do
  SMMD_WINO_WGRAD=$v timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/drv_w${v}.json 2> gpurun_out/drv_w${v}.err || { echo "rc=$?"; tail -5 gpurun_out/drv_w${v}.err; exit 1; }
  python -c "import json; r=json.load(open('gpurun_out/drv_w${v}.json')); print('driver SMMD_WINO_WGRAD=$v', r['value'], r['ms_per_step'])"
done
