# Stride-2 Winograd kernels: standalone parity/timing, their GPU tests + the
# critic-step mirror tests, then the bench with SMMD_WINO_S2=0/1.
set -o pipefail
TAG=${1:-s2}
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 200 python -u tools/wino_s2_bench.py > gpurun_out/${TAG}_bench.txt 2>&1 || { echo "s2 bench rc=$?"; tail -20 gpurun_out/${TAG}_bench.txt; exit 1; }
grep -v amdgpu.ids gpurun_out/${TAG}_bench.txt
timeout -k 10 600 python -u -m pytest tests/test_gpu_wino_s2.py tests/test_gpu_wino.py tests/test_gpu_model.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/${TAG}_tests.txt 2>&1 || { echo "tests rc=$?"; tail -40 gpurun_out/${TAG}_tests.txt; exit 1; }
tail -2 gpurun_out/${TAG}_tests.txt
for i in 1 2; do
  for v in 0 1; do
    SMMD_WINO_S2=$v timeout -k 10 300 python bench.py --steps 30 --warmup 6 --no-cpu-baseline --mmd-sweep 2 --ref-schedule-steps 0 > gpurun_out/${TAG}_bench_s${v}_${i}.json 2> gpurun_out/${TAG}_bench_s${v}_${i}.err || { echo "bench rc=$?"; tail -20 gpurun_out/${TAG}_bench_s${v}_${i}.err; exit 1; }
    python -c "import json; r=json.load(open('gpurun_out/${TAG}_bench_s${v}_${i}.json')); print('SMMD_WINO_S2=$v', r['value'], r['ms_per_step'], r.get('step_ms_by_kind'))"
  done
done
