# Round-6 (r15) evidence on the final tree, every file stamped with the
# library's smmd_source_hash: PMC traffic and executed-FLOP passes (written
# into profiles/r15/ on the box so the bench line embeds them), then the
# default bench line and a kernel trace of the same workload.
# bash tools/gpu_evidence_r15.sh [1 | pmc]
#   pmc: the counter passes only; 1: the bench and the trace only.
# Run them as two gpurun calls (pmc, copy the two JSON files into
# profiles/r15/, then 1): a bench after rocprofv3 --pmc passes in the same
# call ran ~10 % slower on every box tried (5298 / 5304 against 5956 / 5980
# images/s on the same tree), its kernels at the same speed.
set -o pipefail
mkdir -p gpurun_out profiles/r15
export TMPDIR=/tmp
if [ "${1:-0}" != "1" ]; then
bash tools/gpu_pmc.sh ev15 > gpurun_out/ev15_pmc.log 2>&1 || { echo "pmc failed"; tail -20 gpurun_out/ev15_pmc.log; exit 1; }
cp gpurun_out/ev15_traffic.json profiles/r15/pmc_traffic.json
bash tools/gpu_step_pmc.sh ev15s --cycles 2 > gpurun_out/ev15_step.log 2>&1 || { echo "step pmc failed"; tail -20 gpurun_out/ev15_step.log; exit 1; }
python -c "import json;json.load(open('gpurun_out/ev15s_step_flops.json'))" && cp gpurun_out/ev15s_step_flops.json profiles/r15/step_flops_pmc.json
cp profiles/r15/pmc_traffic.json profiles/r15/step_flops_pmc.json gpurun_out/
fi
if [ "${1:-0}" = "pmc" ]; then echo done; exit 0; fi
timeout -k 10 900 python bench.py > gpurun_out/ev15_bench_default.json 2> gpurun_out/ev15_bench_default.err || { echo "bench rc=$?"; tail -20 gpurun_out/ev15_bench_default.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/ev15_bench_default.json'));print(d['value'],d['ms_per_step'],d['roofline']['kernel'],d['roofline']['frac'],d['roofline']['traffic'],d['roofline']['traffic_null_reason'],d['roofline_hot_path']['step']['counters'].get('source'))"
timeout -s KILL 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/ev15_trace -o run -- python tools/step_cycle.py --cycles 2 > gpurun_out/ev15_trace.log 2>&1 || { echo "trace rc=$?"; exit 1; }
find gpurun_out/ev15_trace -name "*kernel_trace.csv" -exec gzip -f {} \;
echo done
