# r04 first pass: GPU tests, the driver's bench invocation, a 60-step bench
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
echo "[r04a] tests"
timeout -k 10 1500 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r04a_tests.txt 2>&1 || { echo "tests rc=$?"; tail -30 gpurun_out/r04a_tests.txt; exit 1; }
tail -3 gpurun_out/r04a_tests.txt
echo "[r04a] bench 20/5"
timeout -k 10 600 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r04a_b20.json 2> gpurun_out/r04a_b20.err || { echo "bench rc=$?"; tail -20 gpurun_out/r04a_b20.err; exit 1; }
head -c 600 gpurun_out/r04a_b20.json; echo
echo "[r04a] bench 60/12"
timeout -k 10 600 python bench.py --steps 60 --warmup 12 --no-cpu-baseline --mmd-sweep 2 > gpurun_out/r04a_b60.json 2> gpurun_out/r04a_b60.err || { echo "bench60 rc=$?"; tail -20 gpurun_out/r04a_b60.err; exit 1; }
head -c 600 gpurun_out/r04a_b60.json; echo
echo "[r04a] done"
