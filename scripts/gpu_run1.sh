set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
python -c "import torch;print(torch.cuda.get_device_name(0), torch.version.hip)" > gpurun_out/env.txt 2>&1
timeout -k 10 600 python -m pytest tests/test_gpu_kernels.py -m gpu -x -q > gpurun_out/pytest_gpu1.log 2>&1
rc=$?
echo "pytest rc=$rc"
tail -30 gpurun_out/pytest_gpu1.log
if [ $rc -eq 0 ]; then
  timeout -k 10 300 python bench.py --steps 50 --warmup 10 > gpurun_out/bench1.log 2>&1; echo "bench rc=$?"; tail -5 gpurun_out/bench1.log
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-graphs --backend torch > gpurun_out/bench1_torch.log 2>&1; echo "bench torch rc=$?"; tail -3 gpurun_out/bench1_torch.log
fi
