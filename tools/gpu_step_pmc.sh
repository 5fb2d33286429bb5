# Executed FLOPs per kernel class over whole 5D+1G cycles (the
# step roofline from counters, not literal MACs) + a kernel trace of the same
# workload for the times: bash tools/gpu_step_pmc.sh TAG [extra step_cycle args]
set -o pipefail
TAG=${1:-r07pmc}
shift
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 60 rocprofv3 -L > gpurun_out/${TAG}_counters.txt 2>&1 || echo "list rc=$?"
grep -o "SQ_INSTS_VALU[A-Z_0-9]*\|SQ_VALU_MFMA_BUSY_CYCLES\|GRBM_GUI_ACTIVE" gpurun_out/${TAG}_counters.txt | sort -u | tr '\n' ' '; echo
timeout -s KILL 300 rocprofv3 --pmc SQ_INSTS_VALU_MFMA_MOPS_F32 SQ_INSTS_VALU_FMA_F32 SQ_INSTS_VALU_ADD_F32 SQ_INSTS_VALU_MUL_F32 SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_VALU_MFMA_F32 GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/${TAG}_pmc -o run -- python tools/step_cycle.py "$@" > gpurun_out/${TAG}_pmc.log 2>&1 || { echo "pmc rc=$?"; tail -5 gpurun_out/${TAG}_pmc.log; exit 1; }
# second counter pass: the hardware's own FLOP tallies (packed ops counted per lane-op)
timeout -s KILL 300 rocprofv3 --pmc SQ_INSTS_VALU_FLOPS_FP32 SQ_INSTS_VALU_FLOPS_FP32_TRANS SQ_INSTS_VALU_MFMA_MOPS_F32 SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/${TAG}_pmc2 -o run -- python tools/step_cycle.py "$@" > gpurun_out/${TAG}_pmc2.log 2>&1 || { echo "pmc2 rc=$?"; tail -5 gpurun_out/${TAG}_pmc2.log; exit 1; }
timeout -s KILL 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_trace -o run -- python tools/step_cycle.py "$@" > gpurun_out/${TAG}_trace.log 2>&1 || { echo "trace rc=$?"; tail -5 gpurun_out/${TAG}_trace.log; exit 1; }
for f in $(find gpurun_out/${TAG}_pmc gpurun_out/${TAG}_pmc2 gpurun_out/${TAG}_trace -name "*counter_collection.csv" -o -name "*kernel_trace.csv"); do gzip -f $f; done
find gpurun_out/${TAG}_pmc gpurun_out/${TAG}_pmc2 gpurun_out/${TAG}_trace -type f | head
python tools/step_flops_pmc.py gpurun_out/${TAG}_pmc gpurun_out/${TAG}_trace 12 gpurun_out/${TAG}_pmc2 > gpurun_out/${TAG}_step_flops.json || echo "post rc=$?"
tail -c 3000 gpurun_out/${TAG}_step_flops.json
echo done
