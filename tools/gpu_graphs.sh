# Step graphs vs eager: the probe at batch 8 / 64 and the bench with --graphs 1
set -o pipefail
TAG=${1:-graphs}
mkdir -p gpurun_out
timeout -k 10 250 python tools/graph_probe.py cifar10 8 > gpurun_out/${TAG}_probe_cifar_b8.txt 2>&1 || { echo probe8 rc=$?; tail -5 gpurun_out/${TAG}_probe_cifar_b8.txt; exit 1; }
timeout -k 10 250 python tools/graph_probe.py imagenet 16 > gpurun_out/${TAG}_probe_imagenet_b16.txt 2>&1 || { echo probe16 rc=$?; exit 1; }
timeout -k 10 250 python tools/graph_probe.py imagenet 64 > gpurun_out/${TAG}_probe_imagenet_b64.txt 2>&1 || { echo probe64 rc=$?; exit 1; }
timeout -k 10 500 python bench.py --graphs 1 --steps 30 --warmup 6 --no-cpu-baseline --mmd-sweep 0 > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err || { echo bench rc=$?; tail -20 gpurun_out/${TAG}_bench.err; exit 1; }
grep -h "ms/step\|^cifar\|^imagenet" gpurun_out/${TAG}_probe_*.txt
python -c "import json; r=json.load(open('gpurun_out/${TAG}_bench.json')); print('bench graphs', r['value'], r['ms_per_step'])"
