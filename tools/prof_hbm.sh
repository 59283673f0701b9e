#!/bin/bash
# rocprofv3 kernel stats + SQ / TCC counter passes of tools/hbm_probe.py (run through gpurun)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/hbm
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/hbm/trace -o run -- python3 tools/hbm_probe.py > gpurun_out/hbm/trace.log 2>&1 || { tail -20 gpurun_out/hbm/trace.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_WAVE_CYCLES --output-format csv -d gpurun_out/hbm/pmc_sq -o run -- python3 tools/hbm_probe.py > gpurun_out/hbm/pmc_sq.log 2>&1 || { tail -20 gpurun_out/hbm/pmc_sq.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE GRBM_GUI_ACTIVE SQ_BUSY_CYCLES SQ_ACTIVE_INST_ANY --output-format csv -d gpurun_out/hbm/pmc_fetch -o run -- python3 tools/hbm_probe.py > gpurun_out/hbm/pmc_fetch.log 2>&1 || { tail -20 gpurun_out/hbm/pmc_fetch.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS --output-format csv -d gpurun_out/hbm/pmc_write -o run -- python3 tools/hbm_probe.py > gpurun_out/hbm/pmc_write.log 2>&1 || { tail -20 gpurun_out/hbm/pmc_write.log; exit 1; }
find gpurun_out/hbm -name "*.csv" | head -20
