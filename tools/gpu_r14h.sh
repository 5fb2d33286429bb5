# Weight-gradient kernels without the operand copies / negations / 64-bit
# chunk division, and the stride-2 sources without SLP: their gpu tests, bit
# for bit against the round-start build, interleaved timing.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
NEW=scaled-mmd-gan_amd/lib/libsmmd_hip.so
timeout -k 10 300 python -u -m pytest tests/test_gpu_wino.py tests/test_gpu_wino_s2.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/r14h_tests.txt 2>&1 || { echo "tests rc=$?"; tail -30 gpurun_out/r14h_tests.txt; exit 1; }
tail -1 gpurun_out/r14h_tests.txt
timeout -k 10 300 python -u tools/lib_bitexact.py tools/hip/v_r14base.so $NEW > gpurun_out/r14h_bitexact.txt 2>&1 || { echo "bitexact rc=$?"; grep -v identical gpurun_out/r14h_bitexact.txt | tail -20; exit 1; }
tail -1 gpurun_out/r14h_bitexact.txt
bash tools/gpu_abn.sh r14h_wg wgrad 2 tools/hip/v_r14base.so tools/hip/v_wgonly.so $NEW || exit 1
bash tools/gpu_abn.sh r14h_s2w s2w 2 tools/hip/v_r14base.so tools/hip/v_wgonly.so $NEW || exit 1
bash tools/gpu_abn.sh r14h_s2 s2 2 tools/hip/v_r14base.so $NEW || exit 1
bash tools/gpu_abn.sh r14h_s2t s2t 2 tools/hip/v_r14base.so $NEW || exit 1
echo done
