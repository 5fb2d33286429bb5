# MIOpen Find experiment: bash tools/gpu_find.sh TAG [bench args]  (GPU box)
set -o pipefail
TAG=${1:-find}
shift || true
EXTRA="$*"      # extra bench.py arguments, e.g. --channels-last 1
mkdir -p gpurun_out/${TAG}_udb
export TMPDIR=/tmp
export MIOPEN_USER_DB_PATH=$PWD/gpurun_out/${TAG}_udb
echo "[find] immediate mode (baseline)"
timeout -k 10 240 python bench.py --steps 30 --warmup 12 --no-cpu-baseline --mmd-sweep 0 --ref-schedule-steps 0 $EXTRA > gpurun_out/${TAG}_imm.json 2> gpurun_out/${TAG}_imm.err || { echo "imm rc=$?"; tail -5 gpurun_out/${TAG}_imm.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/${TAG}_imm.json'));print('immediate', d['value'], d['ms_per_step'])"
echo "[find] cudnn.benchmark"
timeout -k 10 600 python bench.py --steps 30 --warmup 12 --miopen-find 1 --no-cpu-baseline --mmd-sweep 0 --ref-schedule-steps 0 $EXTRA > gpurun_out/${TAG}_find.json 2> gpurun_out/${TAG}_find.err || { echo "find rc=$?"; tail -5 gpurun_out/${TAG}_find.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/${TAG}_find.json'));print('find', d['value'], d['ms_per_step'])"
ls -la gpurun_out/${TAG}_udb
echo "[find] immediate mode with the find db"
timeout -k 10 240 python bench.py --steps 30 --warmup 12 --no-cpu-baseline --mmd-sweep 0 --ref-schedule-steps 0 $EXTRA > gpurun_out/${TAG}_imm2.json 2> gpurun_out/${TAG}_imm2.err || { echo "imm2 rc=$?"; tail -5 gpurun_out/${TAG}_imm2.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/${TAG}_imm2.json'));print('immediate+db', d['value'], d['ms_per_step'])"
