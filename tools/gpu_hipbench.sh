# library-only microbench + its PMC passes: bash tools/gpu_hipbench.sh TAG [pmc]
set -o pipefail
TAG=${1:-hb}
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python tools/hipbench.py --json gpurun_out/${TAG}_time.json > gpurun_out/${TAG}_time.log 2>&1 || { echo "hipbench rc=$?"; tail -20 gpurun_out/${TAG}_time.log; exit 1; }
cat gpurun_out/${TAG}_time.json
if [ "$2" = "pmc" ]; then
  for C in FETCH_SIZE WRITE_SIZE; do
    timeout -k 10 300 rocprofv3 --pmc $C --output-format csv -d gpurun_out/${TAG}_$C -o run -- python tools/hipbench.py --iters 50 > gpurun_out/${TAG}_$C.log 2>&1 || { echo "pmc $C rc=$?"; tail -5 gpurun_out/${TAG}_$C.log; exit 1; }
  done
  python tools/pmc_traffic.py gpurun_out/${TAG}_FETCH_SIZE/run_counter_collection.csv gpurun_out/${TAG}_WRITE_SIZE/run_counter_collection.csv gpurun_out/${TAG}_traffic.json
fi
echo done
