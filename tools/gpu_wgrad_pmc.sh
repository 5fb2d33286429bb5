# SQ counters of the Winograd weight-gradient kernels (one pass, 7 SQ + GRBM):
# where the wave cycles go.  bash tools/gpu_wgrad_pmc.sh TAG
set -o pipefail
TAG=${1:-wgpmc}
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/${TAG}_sq -o run -- python tools/wgrad_probe.py > gpurun_out/${TAG}_sq.log 2>&1 || { echo "sq rc=$?"; tail -5 gpurun_out/${TAG}_sq.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_VALU_MFMA_F32 SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_SALU SQ_VALU_MFMA_COEXEC_CYCLES GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/${TAG}_sq2 -o run -- python tools/wgrad_probe.py > gpurun_out/${TAG}_sq2.log 2>&1 || { echo "sq2 rc=$?"; tail -5 gpurun_out/${TAG}_sq2.log; exit 1; }
timeout -s KILL 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_tr -o run -- python tools/wgrad_probe.py > gpurun_out/${TAG}_tr.log 2>&1 || { echo "trace rc=$?"; tail -5 gpurun_out/${TAG}_tr.log; exit 1; }
python tools/pmc_summary.py gpurun_out/${TAG}_sq gpurun_out/${TAG}_sq2 wgrad
