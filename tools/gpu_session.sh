set -o pipefail
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/t_gpu.log 2>&1 || { tail -30 gpurun_out/t_gpu.log; exit 1; }
tail -1 gpurun_out/t_gpu.log
for i in 1 2; do for nt in 1 0; do
IA_SCREEN_NT=$nt timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/b_nt$nt.json 2> gpurun_out/b_nt$nt.err || { tail -20 gpurun_out/b_nt$nt.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/b_nt$nt.json')); print('nt$nt', round(d['ms_per_step'],1), d['roofline']['screen_avg_us'], d['checks']['checksum'])"
done; done
