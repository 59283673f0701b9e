# PMC passes of the split-f16 screen in the standalone harness (no torch in the process)
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
OUT=$R/gpurun_out/pmc_h16
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
M=${1:-342}
P1="GRBM_GUI_ACTIVE SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU"
P2="SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_WAVES"
i=0
for P in "$P1" "$P2" "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $P --output-format csv -d $OUT/p$i -o pmc -- $R/tools/screen_bench --M $M --reps 2 --rounds 1 > $OUT/p$i.txt 2>&1 || { echo "pass $i failed"; tail -5 $OUT/p$i.txt; exit 1; }
  echo "pass $i done"
done
