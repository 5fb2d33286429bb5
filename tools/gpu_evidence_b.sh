# Round evidence, part B (see tools/gpu_evidence.sh): bash tools/gpu_evidence_b.sh TAG
set -o pipefail
TAG=${1:-ev}
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/${TAG}_bench_driver.json 2> gpurun_out/${TAG}_bench_driver.err || { echo "bench driver rc=$?"; tail -20 gpurun_out/${TAG}_bench_driver.err; exit 1; }
python -c "import json; r=json.load(open('gpurun_out/${TAG}_bench_driver.json')); print('driver', r['value'], r['ms_per_step'])"
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_prof -o run -- python bench.py --steps 30 --warmup 6 --no-cpu-baseline --mmd-sweep 0 --ref-schedule-steps 0 > gpurun_out/${TAG}_prof.json 2> gpurun_out/${TAG}_prof.err || { echo "prof rc=$?"; tail -5 gpurun_out/${TAG}_prof.err; exit 1; }
f=$(find gpurun_out/${TAG}_prof -name "*kernel_stats.csv" | head -1)
python tools/prof_summary.py $f smmd > gpurun_out/${TAG}_prof_smmd.txt && head -30 gpurun_out/${TAG}_prof_smmd.txt
t=$(find gpurun_out/${TAG}_prof -name "*kernel_trace.csv" | head -1)
gzip -f $t
SMMD_DIST_BACKEND=gloo SMMD_SAME_DEVICE=1 timeout -k 10 300 python bench.py --gpus 2 --steps 12 --warmup 6 --no-cpu-baseline --mmd-sweep 2 --ref-schedule-steps 0 > gpurun_out/${TAG}_bench2.json 2> gpurun_out/${TAG}_bench2.err || { echo "bench2 rc=$?"; tail -30 gpurun_out/${TAG}_bench2.err; exit 1; }
timeout -k 10 600 python bench.py --batch 256 --steps 12 --warmup 6 --no-cpu-baseline --mmd-sweep 0 --ref-schedule-steps 6 > gpurun_out/${TAG}_bench_b256.json 2> gpurun_out/${TAG}_bench_b256.err || { echo "b256 rc=$?"; tail -20 gpurun_out/${TAG}_bench_b256.err; exit 1; }
python -c "import json; r=json.load(open('gpurun_out/${TAG}_bench_b256.json')); print('b256', r['value'], r['ms_per_step'])"
echo done
