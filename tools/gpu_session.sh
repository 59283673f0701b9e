# ad-hoc GPU session script (run through gpurun from the repo root)
set -o pipefail
timeout -k 10 300 python -u -m pytest tests/test_gpu_split16.py -x -v -s --timeout 120 --timeout-method thread > gpurun_out/t_split16.log 2>&1 || { tail -40 gpurun_out/t_split16.log; exit 1; }
grep -E "worst|passed|failed" gpurun_out/t_split16.log
timeout -k 10 200 tools/screen_bench --M 32,64,128,256,342 --variants 0x107,0x007,0x207,0x027,0x227 --reps 3 --rounds 3 > gpurun_out/sb_h16s2.txt 2>&1 || { cat gpurun_out/sb_h16s2.txt; exit 1; }
cat gpurun_out/sb_h16s2.txt
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/t_gpu.log 2>&1 || { tail -30 gpurun_out/t_gpu.log; exit 1; }
tail -2 gpurun_out/t_gpu.log
timeout -k 10 300 python bench.py --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/bench_c4_h16s2.json 2> gpurun_out/bench_c4_h16s2.err || { tail gpurun_out/bench_c4_h16s2.err; exit 1; }
cat gpurun_out/bench_c4_h16s2.json
