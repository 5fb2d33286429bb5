# host vs GPU time per step (tools/host_probe.py), then a cProfile of the host side
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u tools/host_probe.py --steps 60 > gpurun_out/host_probe.txt 2>&1 || { echo "probe rc=$?"; tail -20 gpurun_out/host_probe.txt; exit 1; }
grep -v amdgpu.ids gpurun_out/host_probe.txt
timeout -k 10 300 python -u tools/host_probe.py --steps 30 --profile > gpurun_out/host_profile.txt 2>&1 || { echo "profile rc=$?"; tail -20 gpurun_out/host_profile.txt; exit 1; }
head -60 gpurun_out/host_profile.txt | grep -v amdgpu.ids
