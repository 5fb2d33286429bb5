set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python bench.py --steps 30 --warmup 12 > gpurun_out/bench1.log 2> gpurun_out/bench1.err || { echo "bench rc=$?"; exit 1; }
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof1 -o run --output-format csv -- python bench.py --steps 30 --warmup 12 --no-cpu-baseline > gpurun_out/prof1.log 2> gpurun_out/prof1.err || { echo "prof rc=$?"; exit 1; }
echo done
