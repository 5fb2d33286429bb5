# Winograd weight gradient (r11 coalesced form vs the first form): parity tests,
# standalone timing, and the per-kernel split under rocprofv3 (GPU box)
set -o pipefail
TAG=${1:-wg10}
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_wino.py -m gpu -x -q -k wgrad --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/${TAG}_tests.txt 2>&1 || { echo "tests rc=$?"; tail -30 gpurun_out/${TAG}_tests.txt; exit 1; }
tail -1 gpurun_out/${TAG}_tests.txt
timeout -k 10 200 python -u tools/wino_bench.py --iters 10 > gpurun_out/${TAG}_bench.txt 2>&1 || { echo "bench rc=$?"; tail -20 gpurun_out/${TAG}_bench.txt; exit 1; }
grep '^{' gpurun_out/${TAG}_bench.txt | python -c "import sys,json; [print(r['shape'], 'wgrad', round(r.get('wgrad_wino_us',0),1), 'v1', round(r.get('wgrad_v1_us',0),1), 'frac', round(r.get('wgrad_mfma_frac',0),3), 'miopen', round(r.get('wgrad_miopen_us',0),1), 'err', r.get('wgrad_rel_vs_miopen')) for r in map(json.loads, sys.stdin)]"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_prof -o run -- python tools/wino_bench.py --iters 10 > gpurun_out/${TAG}_prof.log 2>&1 || { echo "prof rc=$?"; tail -5 gpurun_out/${TAG}_prof.log; exit 1; }
find gpurun_out/${TAG}_prof -name '*kernel_stats.csv' -exec grep -h "wgrad\|Name" {} \; | cut -c1-200
