# Winograd weight gradient: standalone parity/timing, GPU tests, bench A/B (SMMD_WINO_WGRAD=0/1)
set -o pipefail
TAG=${1:-wg}
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 200 python -u tools/wino_bench.py --iters 10 > gpurun_out/${TAG}_bench.txt 2>&1 || { echo "bench rc=$?"; tail -20 gpurun_out/${TAG}_bench.txt; exit 1; }
grep '^{' gpurun_out/${TAG}_bench.txt | python -c "import sys,json; [print(r['shape'], 'wgrad', round(r.get('wgrad_wino_us',0),1), 'miopen', round(r.get('wgrad_miopen_us',0),1), 'err', r.get('wgrad_rel_vs_miopen')) for r in map(json.loads, sys.stdin)]"
timeout -k 10 600 python -u -m pytest tests/test_gpu_wino.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/${TAG}_tests.txt 2>&1 || { echo "tests rc=$?"; tail -40 gpurun_out/${TAG}_tests.txt; exit 1; }
tail -1 gpurun_out/${TAG}_tests.txt
for i in 1 2; do
  for v in 0 1; do
    SMMD_WINO_WGRAD=$v timeout -k 10 300 python bench.py --steps 30 --warmup 6 --no-cpu-baseline --mmd-sweep 2 --ref-schedule-steps 0 > gpurun_out/${TAG}_bench_w${v}_${i}.json 2> gpurun_out/${TAG}_bench_w${v}_${i}.err || { echo "bench rc=$?"; tail -20 gpurun_out/${TAG}_bench_w${v}_${i}.err; exit 1; }
    python -c "import json; r=json.load(open('gpurun_out/${TAG}_bench_w${v}_${i}.json')); print('SMMD_WINO_WGRAD=$v', r['value'], r['ms_per_step'])"
  done
done
