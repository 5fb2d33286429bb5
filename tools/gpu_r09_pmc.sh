# r09: Winograd GPU tests after the filter-transform change, then the PMC
# traffic passes and the step FLOP counter passes.  bash tools/gpu_r09_pmc.sh TAG
set -o pipefail
TAG=${1:-r09pmc}
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_wino_s2.py tests/test_gpu_wino.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/${TAG}_tests.txt 2>&1 || { echo "tests rc=$?"; tail -30 gpurun_out/${TAG}_tests.txt; exit 1; }
tail -1 gpurun_out/${TAG}_tests.txt
bash tools/gpu_pmc.sh ${TAG}_tr > gpurun_out/${TAG}_tr.out 2>&1 || { echo "pmc traffic failed"; tail -20 gpurun_out/${TAG}_tr.out; exit 1; }
tail -c 1500 gpurun_out/${TAG}_tr.out
bash tools/gpu_step_pmc.sh ${TAG}_st > gpurun_out/${TAG}_st.out 2>&1 || { echo "step pmc failed"; tail -20 gpurun_out/${TAG}_st.out; exit 1; }
tail -c 2500 gpurun_out/${TAG}_st.out
