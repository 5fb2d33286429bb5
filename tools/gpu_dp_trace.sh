# Kernel traces of the one-process step and the world-1 RCCL data-parallel step
# (same bench arguments), for the per-kernel difference: bash tools/gpu_dp_trace.sh TAG
set -o pipefail
TAG=${1:-dptrace}
mkdir -p gpurun_out
export TMPDIR=/tmp
B="--steps 12 --warmup 6 --no-cpu-baseline --mmd-sweep 0 --ref-schedule-steps 0 --instrument-cycles 0"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${TAG}_one -o run --output-format csv -- python bench.py $B > gpurun_out/${TAG}_one.json 2> gpurun_out/${TAG}_one.err || { echo "one rc=$?"; tail -20 gpurun_out/${TAG}_one.err; exit 1; }
echo one done
SMMD_DP_FORCE=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${TAG}_dp -o run --output-format csv -- python bench.py $B > gpurun_out/${TAG}_dp.json 2> gpurun_out/${TAG}_dp.err || { echo "dp rc=$?"; tail -20 gpurun_out/${TAG}_dp.err; exit 1; }
echo dp done
for v in one dp; do
  f=$(find gpurun_out/${TAG}_$v -name '*kernel_trace.csv' | head -1)
  gzip -c "$f" > gpurun_out/${TAG}_${v}_kernel_trace.csv.gz
  rm -f "$f"
done
echo done
