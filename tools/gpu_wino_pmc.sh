# Forward Winograd kernels alone: event times, then SQ counter passes
# (<= 8 SQ counters each).  bash tools/gpu_wino_pmc.sh TAG [3x3|s2]
set -o pipefail
TAG=${1:-wpmc}
ONLY=${2:-}
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 120 python tools/wino_pmc.py --iters 50 ${ONLY:+--only $ONLY} > gpurun_out/${TAG}_times.txt 2>&1 || { echo "times rc=$?"; tail -5 gpurun_out/${TAG}_times.txt; exit 1; }
cat gpurun_out/${TAG}_times.txt
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_INSTS_VALU_MFMA_F32 GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/${TAG}_sq -o run -- python tools/wino_pmc.py --iters 10 ${ONLY:+--only $ONLY} > gpurun_out/${TAG}_sq.log 2>&1 || { echo "sq rc=$?"; tail -5 gpurun_out/${TAG}_sq.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_SALU SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/${TAG}_sq2 -o run -- python tools/wino_pmc.py --iters 10 ${ONLY:+--only $ONLY} > gpurun_out/${TAG}_sq2.log 2>&1 || { echo "sq2 rc=$?"; tail -5 gpurun_out/${TAG}_sq2.log; exit 1; }
python tools/pmc_summary.py gpurun_out/${TAG}_sq gpurun_out/${TAG}_sq2 "smmd::" > gpurun_out/${TAG}_summary.txt
head -200 gpurun_out/${TAG}_summary.txt
