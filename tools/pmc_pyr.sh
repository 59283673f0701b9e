#!/bin/bash
# SQ counters of the pyramid kernels (tools/pyr_sweep.py), two passes
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd /tmp && export TMPDIR=/tmp
P1="GRBM_GUI_ACTIVE SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU"
P2="SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_INSTS_VMEM_RD SQ_WAVES SQ_ACTIVE_INST_SCA"
i=0
for P in "$P1" "$P2"; do
  i=$((i+1))
  PYR_FORMS=1:16,0:16 timeout -s KILL 120 rocprofv3 --pmc $P --output-format csv -d $R/gpurun_out/pmcp$i -o p -- python3 $R/tools/pyr_sweep.py > $R/gpurun_out/pmcp$i.txt 2>&1 || { echo "pass $i failed"; tail -5 $R/gpurun_out/pmcp$i.txt; exit 1; }
done
python3 $R/tools/pmc_summary.py $R/gpurun_out/pmcp*/p_counter_collection.csv > $R/gpurun_out/pmc_pyr.txt
rm -f $R/gpurun_out/pmcp*/p_counter_collection.csv
grep -A18 "k_pyr_strip\|k_pyr_reduce" $R/gpurun_out/pmc_pyr.txt
