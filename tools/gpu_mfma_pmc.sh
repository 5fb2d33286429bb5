# MFMA utilisation of the Gram path from PMC counters: bash tools/gpu_mfma_pmc.sh TAG
set -o pipefail
TAG=${1:-mfma}
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 60 rocprofv3 -L > gpurun_out/${TAG}_counters.txt 2>&1 || echo "list rc=$?"
grep -o "SQ_[A-Z_]*MFMA[A-Z_0-9]*\|GRBM_GUI_ACTIVE\|SQ_BUSY_CYCLES\|SQ_BUSY_CU_CYCLES" gpurun_out/${TAG}_counters.txt | sort -u | head -30
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU_MFMA_MOPS_F32 SQ_INSTS_VALU_MFMA_F32 SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/${TAG}_pmc -o run -- python tools/gram_bench.py --only 2048,1024 --tiles 128 > gpurun_out/${TAG}_pmc.log 2>&1 || { echo "pmc rc=$?"; tail -5 gpurun_out/${TAG}_pmc.log; exit 1; }
ls -R gpurun_out/${TAG}_pmc | head
echo done
