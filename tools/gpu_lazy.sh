# Lazy SN W_eff: its tests, the SN / Winograd / critic-step tests, the bench
set -o pipefail
TAG=${1:-lazy}
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_sn_lazy.py tests/test_gpu_model.py tests/test_gpu_sn_gdirect.py tests/test_gpu_sn_fused.py tests/test_gpu_wino.py tests/test_gpu_wino_s2.py -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/${TAG}_tests.txt 2>&1 || { echo "tests rc=$?"; tail -40 gpurun_out/${TAG}_tests.txt; exit 1; }
tail -1 gpurun_out/${TAG}_tests.txt
bash tools/gpu_round.sh ${TAG} 1
