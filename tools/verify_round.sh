set -o pipefail
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/t_gpu.log 2>&1 || { tail -30 gpurun_out/t_gpu.log; exit 1; }
tail -1 gpurun_out/t_gpu.log
timeout -k 10 300 python -u bench.py > gpurun_out/b_def.json 2> gpurun_out/b_def.err || { tail -20 gpurun_out/b_def.err; exit 1; }
cat gpurun_out/b_def.json
timeout -k 10 900 bash tools/prof_c4.sh ${PROF_TAG:-r01_final} > gpurun_out/prof.log 2>&1 || { tail -20 gpurun_out/prof.log; exit 1; }
echo PROF_OK
