# The whole round evidence in one box acquisition: tests, 60-step bench with
# the CPU baseline, rocprof stats, library PMC passes, batch 256 (gpu_round.sh),
# then the default bench, the driver's command and the 2-rank rehearsal
# (gpu_final.sh).  bash tools/gpu_evidence.sh TAG
set -o pipefail
TAG=${1:-ev}
bash tools/gpu_round.sh ${TAG} || exit 1
bash tools/gpu_final.sh ${TAG}f || exit 1
echo "[evidence] done"
