set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/capture_c4_queries.py > gpurun_out/cap.log 2>&1 || { tail -20 gpurun_out/cap.log; exit 1; }
tail -2 gpurun_out/cap.log
timeout -k 10 900 python -u -m pytest tests/test_gpu_configs.py tests/test_gpu_outputs.py -k "not c4_matcher" -x -v --timeout 600 --timeout-method thread > gpurun_out/t_new.log 2>&1 || { tail -60 gpurun_out/t_new.log; exit 1; }
tail -12 gpurun_out/t_new.log
