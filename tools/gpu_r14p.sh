# Late weight-gradient sums; ReLU mask in the stride-2 transposed conv's epilogue + the zero-free
# create_graph ReLU mask: new tests, the critic-step mirror / wino tests,
# elementwise sources, an interleaved bench A/B of SMMD_RELU_MASK_FUSE.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_relu_mask.py tests/test_gpu_model.py tests/test_gpu_sn_lazy.py tests/test_gpu_fold.py tests/test_gpu_wino_s2.py tests/test_gpu_relupool.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/r14p_tests.txt 2>&1 || { echo "tests rc=$?"; tail -30 gpurun_out/r14p_tests.txt; exit 1; }
tail -1 gpurun_out/r14p_tests.txt
timeout -k 10 300 python -u tools/op_sources.py --top 60 > gpurun_out/r14p_opsrc.txt 2>&1 || { echo "opsrc rc=$?"; tail -20 gpurun_out/r14p_opsrc.txt; exit 1; }
grep "==" gpurun_out/r14p_opsrc.txt
for r in 1 2; do
  for v in 0 1; do
    SMMD_RELU_MASK_FUSE=$v timeout -k 10 400 python bench.py --steps 30 --warmup 5 --no-cpu-baseline --mmd-sweep 0 --ref-schedule-steps 0 > gpurun_out/r14p_ab_${v}_${r}.json 2> gpurun_out/r14p_ab_${v}_${r}.err || { echo "bench rc=$?"; tail -20 gpurun_out/r14p_ab_${v}_${r}.err; exit 1; }
    python -c "import json;d=json.load(open('gpurun_out/r14p_ab_${v}_${r}.json'));print('SMMD_RELU_MASK_FUSE=$v run $r',d['value'],d['ms_per_step'])"
  done
done
echo done
for r in 1 2; do
  for v in 0 1; do
    SMMD_WGRAD_LATE_SUM=$v timeout -k 10 400 python bench.py --steps 30 --warmup 5 --no-cpu-baseline --mmd-sweep 0 --ref-schedule-steps 0 > gpurun_out/r14p_ls_${v}_${r}.json 2> gpurun_out/r14p_ls_${v}_${r}.err || { echo "bench rc=$?"; tail -20 gpurun_out/r14p_ls_${v}_${r}.err; exit 1; }
    python -c "import json;d=json.load(open('gpurun_out/r14p_ls_${v}_${r}.json'));print('SMMD_WGRAD_LATE_SUM=$v run $r',d['value'],d['ms_per_step'])"
  done
done
echo done2
for r in 1 2; do
  for v in 0 1; do
    SMMD_TAIL=$v timeout -k 10 400 python bench.py --steps 30 --warmup 5 --no-cpu-baseline --mmd-sweep 0 --ref-schedule-steps 0 > gpurun_out/r14p_tl_${v}_${r}.json 2> gpurun_out/r14p_tl_${v}_${r}.err || { echo "bench rc=$?"; tail -20 gpurun_out/r14p_tl_${v}_${r}.err; exit 1; }
    python -c "import json;d=json.load(open('gpurun_out/r14p_tl_${v}_${r}.json'));print('SMMD_TAIL=$v run $r',d['value'],d['ms_per_step'])"
  done
done
echo done3
