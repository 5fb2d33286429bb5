# PMC passes (one counter group per pass; no trace domains): bash tools/gpu_pmc.sh TAG
set -o pipefail
TAG=${1:-pmc}
mkdir -p gpurun_out
export TMPDIR=/tmp
for C in FETCH_SIZE WRITE_SIZE; do
  echo "[pmc] $C"
  timeout -k 10 600 rocprofv3 --pmc $C --output-format csv -d gpurun_out/${TAG}_$C -o run -- python bench.py --steps 12 --warmup 12 --no-cpu-baseline > gpurun_out/${TAG}_$C.log 2> gpurun_out/${TAG}_$C.err || { echo "pmc $C rc=$?"; tail -5 gpurun_out/${TAG}_$C.err; exit 1; }
done
ls -R gpurun_out/${TAG}_FETCH_SIZE | head
echo done
