# SQ counters and HBM traffic of the 1x1 kernels at the step's shapes
# (tools/c1_probe.py --pmc launches, one rocprofv3 pass per counter set):
#   bash tools/gpu_c1_pmc.sh TAG
set -o pipefail
TAG=${1:-c1pmc}
mkdir -p gpurun_out
export TMPDIR=/tmp
P1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE"
P2="SQ_INSTS_VALU SQ_INSTS_VALU_MFMA_F32 SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_SALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE"
P3="FETCH_SIZE"
P4="WRITE_SIZE"
i=0
for P in "$P1" "$P2" "$P3" "$P4"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $P --output-format csv -d gpurun_out/${TAG}_p$i -o run -- python tools/c1_probe.py --pmc > gpurun_out/${TAG}_p$i.log 2>&1 || { echo "pass $i rc=$?"; tail -5 gpurun_out/${TAG}_p$i.log; exit 1; }
done
python tools/pmc_summary.py gpurun_out/${TAG}_p1 gpurun_out/${TAG}_p2 gpurun_out/${TAG}_p3 gpurun_out/${TAG}_p4 c1_ > gpurun_out/${TAG}_summary.txt
echo done
