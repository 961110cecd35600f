set -o pipefail
mkdir -p gpurun_out
python -c "import torch;print(torch.cuda.is_available(), torch.cuda.get_device_name(0))" > gpurun_out/env.txt 2>&1
timeout -k 10 600 python -m pytest tests/test_gpu_parity.py -x -q -m gpu > gpurun_out/gpu_parity.log 2>&1
rc=$?
tail -30 gpurun_out/gpu_parity.log
exit $rc
