set -o pipefail
SMMD_GLOBAL_FUSED_LOSS=0 timeout -k 10 100 python -u tools/dbg_global.py > gpurun_out/dbg_global_f0.txt 2>&1; echo "fused0 rc=$?"; grep -E "done|exit|Error|rank" gpurun_out/dbg_global_f0.txt | head
AMD_SERIALIZE_KERNEL=3 timeout -k 10 100 python -u tools/dbg_global.py > gpurun_out/dbg_global_ser.txt 2>&1; echo "ser rc=$?"; grep -v "^  File \"/usr" gpurun_out/dbg_global_ser.txt | head -40
