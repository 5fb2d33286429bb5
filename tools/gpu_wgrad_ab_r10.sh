# Step A/B of the Winograd weight gradient (SMMD_WINO_WGRAD=0/1), interleaved (GPU box)
set -o pipefail
TAG=${1:-wgab10}
mkdir -p gpurun_out
export TMPDIR=/tmp
for i in 1 2; do
  for v in 0 1; do
    SMMD_WINO_WGRAD=$v timeout -k 10 300 python bench.py --steps 30 --warmup 6 --no-cpu-baseline --mmd-sweep 0 --ref-schedule-steps 0 > gpurun_out/${TAG}_w${v}_${i}.json 2> gpurun_out/${TAG}_w${v}_${i}.err || { echo "bench rc=$?"; tail -20 gpurun_out/${TAG}_w${v}_${i}.err; exit 1; }
    python -c "import json; r=json.load(open('gpurun_out/${TAG}_w${v}_${i}.json')); print('SMMD_WINO_WGRAD=$v', r['value'], r['ms_per_step'])"
  done
done
