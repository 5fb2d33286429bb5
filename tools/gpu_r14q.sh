# the late weight-gradient sums' bit-identity test alone
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_model.py -k late_wgrad -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/r14q_tests.txt 2>&1 || { echo "tests rc=$?"; grep -E "Error|assert" gpurun_out/r14q_tests.txt | head -20; exit 1; }
tail -1 gpurun_out/r14q_tests.txt
