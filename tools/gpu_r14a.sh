# Round 5 first GPU pass: the whole gpu suite (new: world-1 RCCL, lazy
# channels_last, stale lazy), the conservative LDS-DMA build bit for bit
# against the shipped one, a bench with the world-1 RCCL group, the default
# driver bench.  bash tools/gpu_r14a.sh
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/r14a_tests.txt 2>&1 || { echo "tests rc=$?"; tail -30 gpurun_out/r14a_tests.txt; exit 1; }
tail -1 gpurun_out/r14a_tests.txt
timeout -k 10 300 python -u tools/lib_bitexact.py scaled-mmd-gan_amd/lib/libsmmd_hip.so scaled-mmd-gan_amd/lib/libsmmd_hip_dmasync.so > gpurun_out/r14a_bitexact.txt 2>&1 || { echo "bitexact rc=$?"; tail -20 gpurun_out/r14a_bitexact.txt; exit 1; }
tail -1 gpurun_out/r14a_bitexact.txt
SMMD_DP_FORCE=1 timeout -k 10 400 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --mmd-sweep 0 --ref-schedule-steps 0 > gpurun_out/r14a_bench_rccl1.json 2> gpurun_out/r14a_bench_rccl1.err || { echo "bench rccl rc=$?"; tail -20 gpurun_out/r14a_bench_rccl1.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/r14a_bench_rccl1.json'));print('rccl1',d['value'],d['ms_per_step'],d['config']['dp_forced'],d['config']['parallelism'])"
timeout -k 10 400 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --mmd-sweep 0 --ref-schedule-steps 0 > gpurun_out/r14a_bench.json 2> gpurun_out/r14a_bench.err || { echo "bench rc=$?"; tail -20 gpurun_out/r14a_bench.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/r14a_bench.json'));print('plain',d['value'],d['ms_per_step'],d['step_ms_by_kind'],d['roofline']['kernel'],d['roofline']['frac'])"
echo done
