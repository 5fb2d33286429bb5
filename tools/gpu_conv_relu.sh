# conv + ReLU epilogue: Winograd GPU tests + critic-step mirror tests, bench A/B (SMMD_CONV_RELU=0/1)
set -o pipefail
TAG=${1:-cr}
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_wino.py tests/test_gpu_wino_s2.py tests/test_gpu_model.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/${TAG}_tests.txt 2>&1 || { echo "tests rc=$?"; tail -40 gpurun_out/${TAG}_tests.txt; exit 1; }
tail -1 gpurun_out/${TAG}_tests.txt
for i in 1 2; do
  for v in 0 1; do
    SMMD_CONV_RELU=$v timeout -k 10 300 python bench.py --steps 30 --warmup 6 --no-cpu-baseline --mmd-sweep 2 --ref-schedule-steps 0 > gpurun_out/${TAG}_bench_r${v}_${i}.json 2> gpurun_out/${TAG}_bench_r${v}_${i}.err || { echo "bench rc=$?"; tail -20 gpurun_out/${TAG}_bench_r${v}_${i}.err; exit 1; }
    python -c "import json; r=json.load(open('gpurun_out/${TAG}_bench_r${v}_${i}.json')); print('SMMD_CONV_RELU=$v', r['value'], r['ms_per_step'])"
  done
done
