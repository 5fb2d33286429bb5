# Find-db refresh for the current conv problems (Winograd path on):
# committed db vs a fresh MIOpen Find (GPU box): bash tools/gpu_find_r10.sh
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
echo "[r10] immediate mode with the committed db"
timeout -k 10 240 python bench.py --steps 30 --warmup 12 --no-cpu-baseline --mmd-sweep 0 --ref-schedule-steps 0 > gpurun_out/r10_committed.json 2> gpurun_out/r10_committed.err || { echo "committed rc=$?"; tail -5 gpurun_out/r10_committed.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/r10_committed.json'));print('committed db', d['value'], d['ms_per_step'])"
bash tools/gpu_find.sh r10find
