# PMC passes (one counter group per pass; no trace domains): bash tools/gpu_pmc.sh TAG
set -o pipefail
TAG=${1:-pmc}
mkdir -p gpurun_out
export TMPDIR=/tmp
for C in FETCH_SIZE WRITE_SIZE; do
  echo "[pmc] $C"
  timeout -k 10 600 rocprofv3 --pmc $C --output-format csv -d gpurun_out/${TAG}_$C -o run -- python tools/step_cycle.py --cycles 2 > gpurun_out/${TAG}_$C.log 2> gpurun_out/${TAG}_$C.err || { echo "pmc $C rc=$?"; tail -5 gpurun_out/${TAG}_$C.err; exit 1; }
done
ls -R gpurun_out/${TAG}_FETCH_SIZE | head
echo done
f1=$(find gpurun_out/${TAG}_FETCH_SIZE -name "*counter_collection.csv" | head -1)
f2=$(find gpurun_out/${TAG}_WRITE_SIZE -name "*counter_collection.csv" | head -1)
python tools/pmc_traffic.py $f1 $f2 gpurun_out/${TAG}_traffic.json > /dev/null && cat gpurun_out/${TAG}_traffic.json
gzip -f $f1 $f2
