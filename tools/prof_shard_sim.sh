cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/ss8 -o ss -- python3 $GRAFT_REPO_ROOT/tools/shard_sim.py 8 > $GRAFT_REPO_ROOT/gpurun_out/ss8.txt 2>&1 || { tail -5 $GRAFT_REPO_ROOT/gpurun_out/ss8.txt; exit 1; }
grep G= $GRAFT_REPO_ROOT/gpurun_out/ss8.txt
head -14 $GRAFT_REPO_ROOT/gpurun_out/ss8/ss_kernel_stats.csv | cut -d, -f1-4
