# SN launch sets: the gpu suite's SN tests, then interleaved sn_bench A/B of
# library builds, then a kernel trace of the shipped build.
#   bash tools/gpu_sn.sh TAG ROUNDS LIB1 LIB2 ...
set -o pipefail
TAG=$1; ROUNDS=$2; shift 2
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider -k "sn or SN or critic_step" > gpurun_out/${TAG}_sntests.txt 2>&1 || { echo "tests rc=$?"; tail -30 gpurun_out/${TAG}_sntests.txt; exit 1; }
tail -1 gpurun_out/${TAG}_sntests.txt
for r in $(seq 1 $ROUNDS); do
  i=0
  for L in "$@"; do
    i=$((i+1))
    SMMD_HIP_LIB=$L timeout -k 10 120 python -u tools/sn_bench.py --iters 200 > gpurun_out/${TAG}_${r}_${i}.txt 2>&1 || { echo "$L rc=$?"; tail -5 gpurun_out/${TAG}_${r}_${i}.txt; exit 1; }
    echo "== round $r $(basename $L)"; tail -1 gpurun_out/${TAG}_${r}_${i}.txt | python -c "import sys,json; d=json.loads(sys.stdin.read()); print(' '.join('%s:%s' % (k, v['avg_us']) for k, v in d.items() if isinstance(v, dict)))"
  done
done
timeout -k 10 180 rocprofv3 --kernel-trace --stats -d gpurun_out/${TAG}_prof -o sn -- python3 tools/sn_bench.py --iters 100 > gpurun_out/${TAG}_prof.log 2>&1 || { echo "prof rc=$?"; tail -20 gpurun_out/${TAG}_prof.log; exit 1; }
echo done
