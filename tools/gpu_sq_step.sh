# SQ counters of every kernel over two whole 5D+1G cycles of the bench
# workload (two passes of <= 8 SQ counters).  bash tools/gpu_sq_step.sh TAG SUBSTR
set -o pipefail
TAG=${1:-sqstep}
SUB=${2:-smmd::}
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -s KILL 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_INSTS_VALU_MFMA_F32 GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/${TAG}_sq -o run -- python tools/step_cycle.py --cycles 1 > gpurun_out/${TAG}_sq.log 2>&1 || { echo "sq rc=$?"; tail -5 gpurun_out/${TAG}_sq.log; exit 1; }
timeout -s KILL 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_SALU SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/${TAG}_sq2 -o run -- python tools/step_cycle.py --cycles 1 > gpurun_out/${TAG}_sq2.log 2>&1 || { echo "sq2 rc=$?"; tail -5 gpurun_out/${TAG}_sq2.log; exit 1; }
for d in gpurun_out/${TAG}_sq gpurun_out/${TAG}_sq2; do find $d -name "*counter_collection.csv" -exec gzip -f {} \; ; done
python tools/pmc_summary.py gpurun_out/${TAG}_sq gpurun_out/${TAG}_sq2 "$SUB" > gpurun_out/${TAG}_summary.txt
head -150 gpurun_out/${TAG}_summary.txt
