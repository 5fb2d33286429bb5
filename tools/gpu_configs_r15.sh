# The other BASELINE configs and the variants of the headline on the final
# tree (stamped lines): bash tools/gpu_configs_r15.sh TAG
#   cifar10 (configs[1]), celebA64 (configs[2]), ImageNet at 256/GPU
#   (configs[4]'s per-GPU batch), the world-1 RCCL data-parallel path, graphs
set -o pipefail
TAG=${1:-cfg15}
mkdir -p gpurun_out
export TMPDIR=/tmp
B="--steps 60 --warmup 12 --no-cpu-baseline --mmd-sweep 0"
run() {
  name=$1; shift
  timeout -k 10 500 "$@" > gpurun_out/${TAG}_$name.json 2> gpurun_out/${TAG}_$name.err || { echo "$name rc=$?"; tail -20 gpurun_out/${TAG}_$name.err; exit 1; }
  python -c "import json; r=json.load(open('gpurun_out/${TAG}_$name.json')); print('$name', r['value'], r['ms_per_step'], r['config'].get('workload'), r['config'].get('parallelism'), r.get('schedule_reference', {}).get('value'))"
}
run cifar10 python bench.py $B --config cifar10
run celebA64 python bench.py $B --config celebA64
run batch256 python bench.py $B --batch 256
run rccl_world1 env SMMD_DP_FORCE=1 python bench.py $B
run nogroup python bench.py $B
run graphs python bench.py $B --graphs 1
echo done
