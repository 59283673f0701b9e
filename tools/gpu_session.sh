# ad-hoc GPU session script (run through gpurun from the repo root)
set -o pipefail
timeout -k 10 400 python -u -m pytest tests/test_gpu_split16.py -x -q -s --timeout 300 --timeout-method thread > gpurun_out/t_split16.log 2>&1 || { tail -40 gpurun_out/t_split16.log; exit 1; }
grep -E "worst|passed|failed" gpurun_out/t_split16.log
timeout -k 10 300 tools/screen_bench --M 128,256,342 --variants 0x007,0x807,0x407,0x4007,0x1007,0x3007,0xb007 --reps 3 --rounds 3 > gpurun_out/sb_h16e.txt 2>&1 || { cat gpurun_out/sb_h16e.txt; exit 1; }
cat gpurun_out/sb_h16e.txt
IA_PRUNE_PROBE=1 timeout -k 10 300 python -u bench.py --steps 1 --warmup 1 > gpurun_out/bench_probe.json 2> gpurun_out/bench_probe.err || { tail -20 gpurun_out/bench_probe.err; exit 1; }
grep prune-probe gpurun_out/bench_probe.err | tail -8
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/t_gpu.log 2>&1 || { tail -30 gpurun_out/t_gpu.log; exit 1; }
tail -2 gpurun_out/t_gpu.log
