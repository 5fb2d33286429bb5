# the step's remaining PyTorch elementwise kernels attributed to their autograd nodes
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python tools/op_sources.py --top 60 > gpurun_out/opsrc_final.txt 2> gpurun_out/opsrc_final.err || { echo "rc=$?"; tail -20 gpurun_out/opsrc_final.err; exit 1; }
echo done
