# Eager vs HIP step graphs on the smaller BASELINE configs (host-bound):
# bash tools/gpu_graphs_cfg.sh TAG
set -o pipefail
TAG=${1:-gcfg}
mkdir -p gpurun_out
export TMPDIR=/tmp
B="--steps 60 --warmup 12 --no-cpu-baseline --mmd-sweep 0 --ref-schedule-steps 0"
for c in cifar10 celebA64; do for g in 0 1; do
  timeout -k 10 400 python bench.py $B --config $c --graphs $g > gpurun_out/${TAG}_${c}_g$g.json 2> gpurun_out/${TAG}_${c}_g$g.err || { echo "$c g$g rc=$?"; tail -20 gpurun_out/${TAG}_${c}_g$g.err; exit 1; }
  python -c "import json; r=json.load(open('gpurun_out/${TAG}_${c}_g$g.json')); print('$c graphs=$g', r['value'], r['ms_per_step'], r.get('step_ms_by_kind'))"
done; done
echo done
