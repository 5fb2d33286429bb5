# tile-kernel timing diagnostics (results of SMMD_TILE_DBG runs are wrong by design)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
G=rbf:64:1,rbf:512:1,rbf:2048:1,rbf:4096:1
for cfg in "0 1024 32" "1 1024 32" "2 1024 32" "6 1024 32" "7 1024 32" "0 512 32" "0 256 32" "0 2048 32" "0 512 64" "0 256 128"; do
  set -- $cfg
  echo "== dbg=$1 blocks=$2 mincpw=$3"
  SMMD_TILE_DBG=$1 SMMD_TILE_BLOCKS=$2 SMMD_TILE_MINCPW=$3 timeout -k 10 120 python tools/mmd_bench.py --grid $G --iters 30 | python -c "import sys,json; print('  '.join('%d:%.1f' % (json.loads(l)['N'], json.loads(l)['us_per_call']) for l in sys.stdin))" || exit 1
done
echo done
