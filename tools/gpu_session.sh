# ad-hoc GPU session script (run through gpurun from the repo root)
set -o pipefail
timeout -k 10 300 python -u -m pytest tests/test_gpu_split16.py -x -q -s --timeout 120 --timeout-method thread > gpurun_out/t_split16.log 2>&1 || { tail -40 gpurun_out/t_split16.log; exit 1; }
grep -E "worst|passed|failed" gpurun_out/t_split16.log
timeout -k 10 200 tools/screen_bench --M 64,128,192,256,342 --variants 0x107,0x007,0x207,0x027 --reps 3 --rounds 3 > gpurun_out/sb_h16s3.txt 2>&1 || { cat gpurun_out/sb_h16s3.txt; exit 1; }
cat gpurun_out/sb_h16s3.txt
bash tools/gpu_pmc.sh 0x007 342 > /dev/null && mv gpurun_out/pmc_h16 gpurun_out/pmc_h16s_342
bash tools/gpu_pmc.sh 0x007 256 > /dev/null && mv gpurun_out/pmc_h16 gpurun_out/pmc_h16s_256
timeout -k 10 300 python bench.py --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/bench_c4_h16s3.json 2> gpurun_out/bench_c4_h16s3.err || { tail gpurun_out/bench_c4_h16s3.err; exit 1; }
cat gpurun_out/bench_c4_h16s3.json
cd /tmp && export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-/root/repo}
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/kt_c4 -o c4 -- python3 $R/bench.py --steps 1 --warmup 1 --no-cpu-baseline > $R/gpurun_out/kt_c4.json 2> $R/gpurun_out/kt_c4.err || { tail $R/gpurun_out/kt_c4.err; exit 1; }
echo kt done
