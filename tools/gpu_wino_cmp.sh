set -o pipefail
mkdir -p gpurun_out
for v in ${VARS:-A E}; do
  timeout -k 10 200 python -u tools/wino_bench.py --lib tools/hip/libwino_$v.so --iters 20 > gpurun_out/wd2_$v.txt 2>&1 || { echo "bench $v rc=$?"; tail -5 gpurun_out/wd2_$v.txt; exit 1; }
  echo "== $v"; grep parity gpurun_out/wd2_$v.txt | head -3; grep '^{' gpurun_out/wd2_$v.txt | python -c "import sys,json; [print(r['shape'], round(r['wino_us'],1), 'miopen', round(r['miopen_fwd_us'],1), 'err', r['fwd_rel_vs_miopen']) for r in map(json.loads, sys.stdin)]"
done
