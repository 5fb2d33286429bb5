mkdir -p gpurun_out
timeout -k 10 300 python tools/conv_probe.py --schedule reference > gpurun_out/cp_ref.txt 2>&1; echo "ref rc=$?"
timeout -k 10 300 python tools/conv_probe.py --schedule lean > gpurun_out/cp_lean.txt 2>&1; echo "lean rc=$?"
timeout -k 10 300 python tools/conv_probe.py --schedule lean --config cifar10 > gpurun_out/cp_cifar.txt 2>&1; echo "cifar rc=$?"
timeout -k 10 300 python tools/conv_probe.py --schedule lean --config celebA64 > gpurun_out/cp_celeba.txt 2>&1; echo "celeba rc=$?"
