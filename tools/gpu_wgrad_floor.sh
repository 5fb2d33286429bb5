set -o pipefail
for r in 1 2; do for L in scaled-mmd-gan_amd/lib/libsmmd_hip.so tools/hip/v_wgnox.so; do
 timeout -k 10 120 python -u tools/wino_pmc.py --lib $L --iters 30 --only wgrad > gpurun_out/wg_$(basename $L .so)_$r.txt 2>&1 || { echo fail; tail -5 gpurun_out/wg_$(basename $L .so)_$r.txt; exit 1; }
 echo "== $L"; tail -1 gpurun_out/wg_$(basename $L .so)_$r.txt | python -c "import sys,json; d=json.loads(sys.stdin.read()); [print(k, v['us'], v.get('mfma_frac')) for k, v in d.items() if isinstance(v, dict)]"
done; done
