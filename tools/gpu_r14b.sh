# the sliced stride-2 kernels: bit for bit against the round-start build and
# the conservative DMA build, interleaved timing with slot variants, then the
# gpu suite.  bash tools/gpu_r14b.sh
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
NEW=scaled-mmd-gan_amd/lib/libsmmd_hip.so
timeout -k 10 300 python -u tools/lib_bitexact.py tools/hip/v_r13base.so $NEW > gpurun_out/r14b_bitexact_base.txt 2>&1 || { echo "bitexact base rc=$?"; tail -20 gpurun_out/r14b_bitexact_base.txt; exit 1; }
tail -1 gpurun_out/r14b_bitexact_base.txt
timeout -k 10 300 python -u tools/lib_bitexact.py $NEW scaled-mmd-gan_amd/lib/libsmmd_hip_dmasync.so > gpurun_out/r14b_bitexact_dma.txt 2>&1 || { echo "bitexact dma rc=$?"; tail -20 gpurun_out/r14b_bitexact_dma.txt; exit 1; }
tail -1 gpurun_out/r14b_bitexact_dma.txt
bash tools/gpu_abn.sh r14b_s2 s2 2 tools/hip/v_r13base.so $NEW tools/hip/v_slot16.so tools/hip/v_slot24.so tools/hip/v_slot28.so || exit 1
bash tools/gpu_abn.sh r14b_s2t s2t 2 tools/hip/v_r13base.so $NEW tools/hip/v_slot16.so tools/hip/v_slot24.so tools/hip/v_slot28.so || exit 1
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/r14b_tests.txt 2>&1 || { echo "tests rc=$?"; tail -30 gpurun_out/r14b_tests.txt; exit 1; }
tail -1 gpurun_out/r14b_tests.txt
echo done
