# stride-2 kernels at reduction-slice targets 256 / 512 / 1024 workgroups
set -o pipefail
mkdir -p gpurun_out
for t in 512 256 1024; do
  SMMD_S2_BLOCKS=$t timeout -k 10 200 python -u tools/wino_s2_bench.py > gpurun_out/s2sl_$t.txt 2>&1 || { echo "rc=$?"; tail -5 gpurun_out/s2sl_$t.txt; exit 1; }
  echo "== target $t"; grep '^{' gpurun_out/s2sl_$t.txt | python -c "import sys,json; [print(r['shape'], r['wino_us'], r['dgrad_wino_us']) for r in map(json.loads, sys.stdin)]"
done
