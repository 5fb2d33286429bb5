# Winograd kernel diagnosis: timing of variant libraries (tools/hip/libwino_*.so,
# built from csrc/smmd_wino.hip with parts removed) and one SQ counter pass
# over the product kernel.  bash tools/gpu_wino_diag.sh TAG
set -o pipefail
TAG=${1:-wdiag}
mkdir -p gpurun_out
export TMPDIR=/tmp
for v in A B C D; do
  timeout -k 10 200 python -u tools/wino_bench.py --lib tools/hip/libwino_$v.so --iters 10 > gpurun_out/${TAG}_$v.txt 2>&1 || { echo "bench $v rc=$?"; tail -5 gpurun_out/${TAG}_$v.txt; exit 1; }
  echo "== $v"; grep '^{' gpurun_out/${TAG}_$v.txt | python -c "import sys,json; [print(r['shape'], round(r['wino_us'],1), 'miopen', round(r['miopen_fwd_us'],1)) for r in map(json.loads, sys.stdin)]"
done
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/${TAG}_pmc -o run -- python tools/wino_bench.py --lib tools/hip/libwino_A.so --iters 3 > gpurun_out/${TAG}_pmc.log 2>&1 || { echo "pmc rc=$?"; tail -5 gpurun_out/${TAG}_pmc.log; exit 1; }
f=$(find gpurun_out/${TAG}_pmc -name "*counter_collection.csv" | head -1)
python - "$f" <<'PY'
import csv, sys, collections
rows = list(csv.DictReader(open(sys.argv[1])))
acc = collections.defaultdict(lambda: collections.defaultdict(list))
for r in rows:
    k = r['Kernel_Name']
    if 'wino_conv' not in k:
        continue
    key = (k[:40], r.get('Grid_Size', r.get('Grid_Size_X', '')))
    acc[key][r['Counter_Name']].append(float(r['Counter_Value']))
for key, d in acc.items():
    print(key, {c: round(sum(v) / len(v)) for c, v in d.items()})
PY
gzip -f $f
