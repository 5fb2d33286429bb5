# single-output linear node (snops._LinOut): model tests + interleaved bench A/B
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_model.py tests/test_gpu_dist.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/linnode_tests.txt 2>&1 || { echo "tests rc=$?"; tail -30 gpurun_out/linnode_tests.txt; exit 1; }
tail -1 gpurun_out/linnode_tests.txt
for r in 1 2; do
  for v in 1 0; do
    SMMD_LINEAR_NODE=$v timeout -k 10 400 python bench.py --steps 40 --warmup 5 --no-cpu-baseline --mmd-sweep 0 --ref-schedule-steps 0 > gpurun_out/linnode_${v}_${r}.json 2> gpurun_out/linnode_${v}_${r}.err || { echo "bench rc=$?"; tail -20 gpurun_out/linnode_${v}_${r}.err; exit 1; }
    python -c "import json;d=json.load(open('gpurun_out/linnode_${v}_${r}.json'));print('SMMD_LINEAR_NODE=$v run $r',d['value'],d['ms_per_step'])"
  done
done
echo done
