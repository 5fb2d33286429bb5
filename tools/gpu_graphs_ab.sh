set -o pipefail
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_model.py -k "graphs" > gpurun_out/r15c_tests.txt 2>&1 || { tail -30 gpurun_out/r15c_tests.txt; exit 1; }
tail -4 gpurun_out/r15c_tests.txt
bash tools/gpu_ab.sh r15c_graphs "--steps 30 --warmup 6 --mmd-sweep 0 --ref-schedule-steps 0 --graphs 0" "--steps 30 --warmup 6 --mmd-sweep 0 --ref-schedule-steps 0 --graphs 1" "--steps 30 --warmup 6 --mmd-sweep 0 --ref-schedule-steps 0 --graphs 0" "--steps 30 --warmup 6 --mmd-sweep 0 --ref-schedule-steps 0 --graphs 1"
