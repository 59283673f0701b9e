#!/bin/bash
# kernel durations of ia_pyr_reduce_f64's forms (tools/pyr_sweep.py under rocprofv3)
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/pyr2 -o pyr -- python3 $R/tools/pyr_sweep.py > $R/gpurun_out/pyr2.txt 2>&1 || { tail -5 $R/gpurun_out/pyr2.txt; exit 1; }
cut -d, -f1-4 $R/gpurun_out/pyr2/pyr_kernel_stats.csv | head -12
rm -f $R/gpurun_out/pyr2/pyr_kernel_trace.csv
