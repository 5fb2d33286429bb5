# usage: bash tools/gpu_all.sh TAG   (run on the GPU box via gpurun)
set -o pipefail
TAG=${1:-run}
mkdir -p gpurun_out
export TMPDIR=/tmp
echo "[gpu_all] tests" 
timeout -k 10 900 python -m pytest tests -q -m gpu > gpurun_out/${TAG}_tests.log 2>&1 || { echo "tests rc=$?"; tail -30 gpurun_out/${TAG}_tests.log; exit 1; }
tail -2 gpurun_out/${TAG}_tests.log
echo "[gpu_all] bench"
timeout -k 10 900 python bench.py --steps 60 --warmup 12 > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err || { echo "bench rc=$?"; tail -20 gpurun_out/${TAG}_bench.err; exit 1; }
cat gpurun_out/${TAG}_bench.json
echo "[gpu_all] rocprof"
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/${TAG}_prof -o run --output-format csv -- python bench.py --steps 30 --warmup 12 --no-cpu-baseline --mmd-sweep 0 --ref-schedule-steps 0 > gpurun_out/${TAG}_prof.log 2> gpurun_out/${TAG}_prof.err || { echo "prof rc=$?"; tail -20 gpurun_out/${TAG}_prof.err; exit 1; }
if [ "$2" = "pmc" ]; then
  echo "[gpu_all] pmc (library-only microbench)"
  bash tools/gpu_hipbench.sh ${TAG}_hb pmc > gpurun_out/${TAG}_hb.log 2>&1 || { echo "pmc rc=$?"; tail -5 gpurun_out/${TAG}_hb.log; exit 1; }
fi
echo "[gpu_all] done"
