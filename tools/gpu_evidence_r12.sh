# Round-4 (r12) evidence on the final tree, every file stamped with the
# library's smmd_source_hash: PMC traffic and executed-FLOP passes (written
# into profiles/r12/ on the box so the bench line embeds them), then the
# default bench line and a kernel trace of the same workload.
# bash tools/gpu_evidence_r11.sh [skip_pmc]
set -o pipefail
mkdir -p gpurun_out profiles/r12
export TMPDIR=/tmp
if [ "${1:-0}" != "1" ]; then
bash tools/gpu_pmc.sh ev12 > gpurun_out/ev12_pmc.log 2>&1 || { echo "pmc failed"; tail -20 gpurun_out/ev12_pmc.log; exit 1; }
cp gpurun_out/ev12_traffic.json profiles/r12/pmc_traffic.json
bash tools/gpu_step_pmc.sh ev12s --cycles 2 > gpurun_out/ev12_step.log 2>&1 || { echo "step pmc failed"; tail -20 gpurun_out/ev12_step.log; exit 1; }
python -c "import json;json.load(open('gpurun_out/ev12s_step_flops.json'))" && cp gpurun_out/ev12s_step_flops.json profiles/r12/step_flops_pmc.json
cp profiles/r12/pmc_traffic.json profiles/r12/step_flops_pmc.json gpurun_out/
fi
timeout -k 10 900 python bench.py > gpurun_out/ev12_bench_default.json 2> gpurun_out/ev12_bench_default.err || { echo "bench rc=$?"; tail -20 gpurun_out/ev12_bench_default.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/ev12_bench_default.json'));print(d['value'],d['ms_per_step'],d['roofline']['kernel'],d['roofline']['frac'],d['roofline']['traffic'],d['roofline']['traffic_null_reason'],d['roofline_hot_path']['step']['counters'].get('source'))"
timeout -s KILL 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/ev12_trace -o run -- python tools/step_cycle.py --cycles 2 > gpurun_out/ev12_trace.log 2>&1 || { echo "trace rc=$?"; exit 1; }
find gpurun_out/ev12_trace -name "*kernel_trace.csv" -exec gzip -f {} \;
echo done
