set -o pipefail
timeout -k 10 400 python -u -m pytest tests/test_gpu_split16.py -x -q -s --timeout 300 --timeout-method thread -k "forms" > gpurun_out/t_split16.log 2>&1 || { tail -40 gpurun_out/t_split16.log; exit 1; }
grep -E "passed|failed" gpurun_out/t_split16.log
timeout -k 10 300 tools/screen_bench --M 160,192,256,288,320,342 --variants 0x007,0x40007 --reps 3 --rounds 5 > gpurun_out/sb_h16b.txt 2>&1 || { cat gpurun_out/sb_h16b.txt; exit 1; }
cat gpurun_out/sb_h16b.txt
