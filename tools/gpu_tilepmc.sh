# PMC counters of the tile kernel (one pass per counter set, no trace domains)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
for N in 512 2048; do
  timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_SMEM --output-format csv -d gpurun_out/tpmc_$N -o run -- python tools/mmd_bench.py --grid rbf:$N:1 --iters 10 > gpurun_out/tpmc_$N.log 2>&1 || { echo "pmc rc=$?"; tail -5 gpurun_out/tpmc_$N.log; exit 1; }
  timeout -s KILL 90 rocprofv3 --pmc GRBM_GUI_ACTIVE GRBM_COUNT SQ_INSTS_SALU SQ_ACTIVE_INST_SCA SQ_INST_CYCLES_SMEM SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_INSTS_LDS --output-format csv -d gpurun_out/tpmc2_$N -o run -- python tools/mmd_bench.py --grid rbf:$N:1 --iters 10 > gpurun_out/tpmc2_$N.log 2>&1 || { echo "pmc2 rc=$?"; tail -5 gpurun_out/tpmc2_$N.log; exit 1; }
done
python - <<'PY'
import csv, glob
from collections import defaultdict
for d in sorted(glob.glob('gpurun_out/tpmc*_*')):
    for f in glob.glob(d + '/*counter_collection.csv'):
        acc = defaultdict(list)
        for r in csv.DictReader(open(f)):
            if 'tile_kernel' not in r['Kernel_Name']:
                continue
            acc[r['Counter_Name']].append(float(r['Counter_Value']))
        print(d, {k: round(sum(v) / len(v)) for k, v in acc.items()})
PY
echo done
