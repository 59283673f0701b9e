set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_split16.py tests/test_gpu_parity.py tests/test_gpu_configs.py -x -v --timeout 300 --timeout-method thread > gpurun_out/t_db.log 2>&1 || { tail -40 gpurun_out/t_db.log; exit 1; }
tail -3 gpurun_out/t_db.log
timeout -k 10 300 python -u -c "
import sys, json; sys.path.insert(0,'.'); import bench, torch
print(json.dumps(bench.hbm_kernels(torch.device('cuda:0')), indent=1))" > gpurun_out/hbm.json 2>&1 || { tail -20 gpurun_out/hbm.json; exit 1; }
cat gpurun_out/hbm.json
