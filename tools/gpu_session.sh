set -o pipefail
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/t_gpu.log 2>&1 || { tail -30 gpurun_out/t_gpu.log; exit 1; }
tail -1 gpurun_out/t_gpu.log
timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/b_g.json 2> gpurun_out/b_g.err || { tail -20 gpurun_out/b_g.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/b_g.json')); print('gather2', round(d['ms_per_step'],1), round(d['roofline']['screen_avg_us'],1), round(d['roofline']['frac'],4), d['checks']['checksum'])"
