# kernel time of the MMD launch at the configs' small sizes: single workgroup vs grid
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
for S in 1 0; do
  SMMD_TILE_SMALL=$S timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/mmdsmall_$S -o run -- python tools/mmd_bench.py --iters 200 --grid rbf:64:1,rbf:128:1,mix_rq:64:1,mix_rbf:64:1 > gpurun_out/mmdsmall_$S.log 2>&1 || { echo "rc=$?"; tail -5 gpurun_out/mmdsmall_$S.log; exit 1; }
  echo "SMMD_TILE_SMALL=$S"; grep -h "us_per_call" gpurun_out/mmdsmall_$S.log | cut -c1-120
  F=$(find gpurun_out/mmdsmall_$S -name '*kernel_stats.csv' | head -1); grep -h "mmd2" "$F" | cut -d, -f1-4 | cut -c1-160
done
