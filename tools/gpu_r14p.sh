# This round's elementwise fusions (ReLU mask in the stride-2 transposed conv,
# zero-free create_graph ReLU mask, late weight-gradient sums, the critic tail,
# the generator's gradient gather): their tests, the critic-step mirror and
# the wino tests, the elementwise sources, and bench A/Bs -- everything off vs
# on (interleaved, twice), then each switch off alone.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_relu_mask.py tests/test_gpu_model.py tests/test_gpu_sn_lazy.py tests/test_gpu_fold.py tests/test_gpu_wino_s2.py tests/test_gpu_relupool.py tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/r14p_tests.txt 2>&1 || { echo "tests rc=$?"; tail -30 gpurun_out/r14p_tests.txt; exit 1; }
tail -1 gpurun_out/r14p_tests.txt
timeout -k 10 300 python -u tools/op_sources.py --top 60 > gpurun_out/r14p_opsrc.txt 2>&1 || { echo "opsrc rc=$?"; tail -20 gpurun_out/r14p_opsrc.txt; exit 1; }
grep "==" gpurun_out/r14p_opsrc.txt
OFF="SMMD_RELU_MASK_FUSE=0 SMMD_WGRAD_LATE_SUM=0 SMMD_TAIL=0 SMMD_GRAD_GATHER=0"
run() {  # tag env...
  local tag=$1; shift
  env "$@" timeout -k 10 400 python bench.py --steps 30 --warmup 5 --no-cpu-baseline --mmd-sweep 0 --ref-schedule-steps 0 > gpurun_out/r14p_${tag}.json 2> gpurun_out/r14p_${tag}.err || { echo "bench $tag rc=$?"; tail -20 gpurun_out/r14p_${tag}.err; return 1; }
  python -c "import json;d=json.load(open('gpurun_out/r14p_${tag}.json'));print('$tag',d['value'],d['ms_per_step'])"
}
for r in 1 2; do
  run alloff_$r $OFF || exit 1
  run allon_$r X=1 || exit 1
done
run nomask SMMD_RELU_MASK_FUSE=0 || exit 1
run nolate SMMD_WGRAD_LATE_SUM=0 || exit 1
run notail SMMD_TAIL=0 || exit 1
run nogather SMMD_GRAD_GATHER=0 || exit 1
echo done
