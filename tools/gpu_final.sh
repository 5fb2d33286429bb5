# 2-rank rehearsal (gloo on one GPU) of the global mode's exchange + buckets,
# then the default bench (no flags: N=1, cpu baseline, full MMD sweep) and the
# driver's own command line.  bash tools/gpu_final.sh TAG
set -o pipefail
TAG=${1:-final}
mkdir -p gpurun_out
export TMPDIR=/tmp
SMMD_DIST_BACKEND=gloo SMMD_SAME_DEVICE=1 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 2 --steps 6 --warmup 6 --no-cpu-baseline --mmd-sweep 2 --ref-schedule-steps 0 > gpurun_out/${TAG}_bench2.json 2> gpurun_out/${TAG}_bench2.err || { echo "bench2 rc=$?"; tail -30 gpurun_out/${TAG}_bench2.err; exit 1; }
python -c "import json; r=json.loads([l for l in open('gpurun_out/${TAG}_bench2.json') if l.startswith('{')][-1]); print('2 ranks', r['value'], r['n_gpus'], r['ms_per_step'])"
timeout -k 10 900 python bench.py > gpurun_out/${TAG}_bench_default.json 2> gpurun_out/${TAG}_bench_default.err || { echo "bench rc=$?"; tail -20 gpurun_out/${TAG}_bench_default.err; exit 1; }
python -c "import json; r=json.load(open('gpurun_out/${TAG}_bench_default.json')); print('default', r['value'], r['ms_per_step'], r['cpu_baseline']['value'], list(r['cpu_baseline'].get('components', {})))"
timeout -k 10 600 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/${TAG}_bench_driver.json 2> gpurun_out/${TAG}_bench_driver.err || { echo "bench driver rc=$?"; tail -20 gpurun_out/${TAG}_bench_driver.err; exit 1; }
python -c "import json; r=json.load(open('gpurun_out/${TAG}_bench_driver.json')); print('driver', r['value'], r['ms_per_step'])"
echo done
