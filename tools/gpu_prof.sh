# Kernel-trace stats + the two PMC passes of the bench, and the per-entry-point
# traffic summary: bash tools/gpu_prof.sh TAG   (outputs under gpurun_out/TAG_*)
set -o pipefail
TAG=${1:-prof}
mkdir -p gpurun_out
export TMPDIR=/tmp
echo "[prof] kernel trace"
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_kt -o run -- python bench.py --steps 20 --warmup 5 --no-cpu-baseline --mmd-sweep 0 > gpurun_out/${TAG}_kt_bench.json 2> gpurun_out/${TAG}_kt.err || { echo "kt rc=$?"; tail -5 gpurun_out/${TAG}_kt.err; exit 1; }
for C in FETCH_SIZE WRITE_SIZE; do
  echo "[prof] pmc $C"
  timeout -k 10 600 rocprofv3 --pmc $C --output-format csv -d gpurun_out/${TAG}_$C -o run -- python bench.py --steps 12 --warmup 12 --no-cpu-baseline --instrument-cycles 0 --mmd-sweep 0 --ref-schedule-steps 0 > gpurun_out/${TAG}_$C.log 2> gpurun_out/${TAG}_$C.err || { echo "pmc $C rc=$?"; tail -5 gpurun_out/${TAG}_$C.err; exit 1; }
done
F=$(find gpurun_out/${TAG}_FETCH_SIZE -name '*counter_collection.csv' | head -1)
W=$(find gpurun_out/${TAG}_WRITE_SIZE -name '*counter_collection.csv' | head -1)
python tools/pmc_traffic.py "$F" "$W" gpurun_out/${TAG}_pmc_traffic.json > /dev/null || exit 1
S=$(find gpurun_out/${TAG}_kt -name '*kernel_stats.csv' | head -1)
cp "$S" gpurun_out/${TAG}_kernel_stats.csv
echo done
