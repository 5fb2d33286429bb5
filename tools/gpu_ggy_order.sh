set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python tools/ggy_order.py > gpurun_out/ggy_order.txt 2> gpurun_out/ggy_order.err || { echo "rc=$?"; tail -20 gpurun_out/ggy_order.err; exit 1; }
cat gpurun_out/ggy_order.txt
