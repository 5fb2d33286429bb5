# slot variants of the sliced stride-2 kernels (interleaved), then the gpu suite
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
NEW=scaled-mmd-gan_amd/lib/libsmmd_hip.so
bash tools/gpu_abn.sh r14c_s2 s2 2 tools/hip/v_r13base.so $NEW tools/hip/v_slot16.so tools/hip/v_slot24.so tools/hip/v_slot28.so || exit 1
bash tools/gpu_abn.sh r14c_s2t s2t 2 tools/hip/v_r13base.so $NEW tools/hip/v_slot16.so tools/hip/v_slot24.so tools/hip/v_slot28.so || exit 1
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/r14c_tests.txt 2>&1 || { echo "tests rc=$?"; tail -30 gpurun_out/r14c_tests.txt; exit 1; }
tail -1 gpurun_out/r14c_tests.txt
echo done
