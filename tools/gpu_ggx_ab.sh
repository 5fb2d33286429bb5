# SMMD_GGX_MASK_FUSE interleaved bench A/B only (three rounds, order alternating)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
for r in 1 2 3; do
  for v in 1 0; do
    SMMD_GGX_MASK_FUSE=$v timeout -k 10 400 python bench.py --steps 40 --warmup 5 --no-cpu-baseline --mmd-sweep 0 --ref-schedule-steps 0 > gpurun_out/ggxab_${v}_${r}.json 2> gpurun_out/ggxab_${v}_${r}.err || { echo "bench rc=$?"; tail -20 gpurun_out/ggxab_${v}_${r}.err; exit 1; }
    python -c "import json;d=json.load(open('gpurun_out/ggxab_${v}_${r}.json'));print('SMMD_GGX_MASK_FUSE=$v run $r',d['value'],d['ms_per_step'])"
  done
done
echo done
