set -o pipefail
timeout -k 10 400 python -u -m pytest tests/test_gpu_split16.py -x -q -s --timeout 300 --timeout-method thread -k "forms" > gpurun_out/t_split16.log 2>&1 || { tail -40 gpurun_out/t_split16.log; exit 1; }
grep -E "passed|failed" gpurun_out/t_split16.log
timeout -k 10 300 tools/screen_bench --M 160,192,224 --variants 0x207,0x007 --reps 3 --rounds 5 > gpurun_out/sb_h16c2.txt 2>&1 || { cat gpurun_out/sb_h16c2.txt; exit 1; }
cat gpurun_out/sb_h16c2.txt
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/t_gpu.log 2>&1 || { tail -30 gpurun_out/t_gpu.log; exit 1; }
tail -1 gpurun_out/t_gpu.log
for bal in 1 0; do
IA_SCREEN_BAL=$bal timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/b_bal$bal.json 2> gpurun_out/b_bal$bal.err || { tail -20 gpurun_out/b_bal$bal.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/b_bal$bal.json')); print('bal$bal', round(d['ms_per_step'],1), round(d['roofline']['screen_avg_us'],1), round(d['roofline']['frac'],4), d['checks']['checksum'])"
done
