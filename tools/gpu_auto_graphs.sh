# bench.py's default (auto graphs) on the three single-GPU configs: bash tools/gpu_auto_graphs.sh TAG
set -o pipefail
TAG=${1:-auto}
mkdir -p gpurun_out
export TMPDIR=/tmp
B="--steps 60 --warmup 12 --no-cpu-baseline --mmd-sweep 0"
for c in imagenet cifar10 celebA64; do
  timeout -k 10 500 python bench.py $B --config $c > gpurun_out/${TAG}_$c.json 2> gpurun_out/${TAG}_$c.err || { echo "$c rc=$?"; tail -20 gpurun_out/${TAG}_$c.err; exit 1; }
  python -c "import json; r=json.load(open('gpurun_out/${TAG}_$c.json')); print('$c', r['value'], r['ms_per_step'], r['config'].get('step_graphs'), r['config'].get('step_graphs_probe'))"
done
echo done
