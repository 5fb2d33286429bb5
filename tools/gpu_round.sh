# Round evidence on one box: bash tools/gpu_round.sh TAG
#   GPU tests, the default bench line, its rocprof kernel stats, the
#   library-only PMC passes, and a batch-256 bench line (BASELINE configs[4]
#   per GPU)
set -o pipefail
TAG=${1:-round}
bash tools/gpu_all.sh ${TAG} pmc || exit 1
echo "[round] batch 256"
timeout -k 10 600 python bench.py --batch 256 --steps 24 --warmup 8 --no-cpu-baseline --mmd-sweep 0 --ref-schedule-steps 0 > gpurun_out/${TAG}_b256.json 2> gpurun_out/${TAG}_b256.err || { echo "b256 rc=$?"; tail -20 gpurun_out/${TAG}_b256.err; exit 1; }
head -c 300 gpurun_out/${TAG}_b256.json
echo
echo "[round] done"
