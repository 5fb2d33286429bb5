# Final evidence on the tree: GPU tests, default bench, then part B (driver, rocprof, 2-rank, batch 256)
set -o pipefail
TAG=${1:-r09f}
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/${TAG}_gpu_tests.txt 2>&1 || { echo "tests rc=$?"; tail -30 gpurun_out/${TAG}_gpu_tests.txt; exit 1; }
tail -1 gpurun_out/${TAG}_gpu_tests.txt
timeout -k 10 400 python bench.py > gpurun_out/${TAG}_bench_default.json 2> gpurun_out/${TAG}_bench_default.err || { echo "bench rc=$?"; tail -20 gpurun_out/${TAG}_bench_default.err; exit 1; }
python -c "import json; r=json.load(open('gpurun_out/${TAG}_bench_default.json')); print('default', r['value'], r['ms_per_step'], r['roofline']['kernel'] if 'kernel' in r['roofline'] else '', r['roofline']['frac'])"
bash tools/gpu_evidence_b.sh ${TAG}
