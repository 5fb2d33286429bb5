# Add the find results of another bench shape to the committed MIOpen find db:
#   bash tools/gpu_find_merge.sh TAG "--batch 256"     (GPU box)
# Starts from a copy of scaled-mmd-gan_amd/miopen_db/, runs the bench with
# cudnn.benchmark on the given args (MIOpen appends the new problems), then the
# same bench in immediate mode with the merged db and with the committed one.
set -o pipefail
TAG=${1:-fm}
ARGS=${2:-"--batch 256"}
mkdir -p gpurun_out/${TAG}_udb
export TMPDIR=/tmp
cp scaled-mmd-gan_amd/miopen_db/*.txt gpurun_out/${TAG}_udb/
B="timeout -k 10 700 python bench.py --steps 24 --warmup 8 --no-cpu-baseline --mmd-sweep 0 --ref-schedule-steps 0 $ARGS"
echo "[find-merge] immediate, committed db"
$B > gpurun_out/${TAG}_imm.json 2> gpurun_out/${TAG}_imm.err || { echo "imm rc=$?"; tail -5 gpurun_out/${TAG}_imm.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/${TAG}_imm.json'));print('immediate', d['value'], d['ms_per_step'])"
echo "[find-merge] cudnn.benchmark into the copy"
MIOPEN_USER_DB_PATH=$PWD/gpurun_out/${TAG}_udb $B --miopen-find 1 > gpurun_out/${TAG}_find.json 2> gpurun_out/${TAG}_find.err || { echo "find rc=$?"; tail -5 gpurun_out/${TAG}_find.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/${TAG}_find.json'));print('find', d['value'], d['ms_per_step'])"
echo "[find-merge] immediate, merged db"
MIOPEN_USER_DB_PATH=$PWD/gpurun_out/${TAG}_udb $B > gpurun_out/${TAG}_imm2.json 2> gpurun_out/${TAG}_imm2.err || { echo "imm2 rc=$?"; tail -5 gpurun_out/${TAG}_imm2.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/${TAG}_imm2.json'));print('immediate+merged', d['value'], d['ms_per_step'])"
wc -l gpurun_out/${TAG}_udb/*.txt
