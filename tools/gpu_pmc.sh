# PMC passes over a command (default: bench.py, the headline encode), one
# counter group per run; summarise with tools/pmc_summary.py <kernel-substring> <dir>.
set -o pipefail
export TMPDIR=/tmp
OUT=${PMC_OUT:-gpurun_out/pmc}
mkdir -p $OUT
i=0
for ctrs in "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVES GRBM_GUI_ACTIVE" \
            "SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_WAVE_CYCLES SQ_BUSY_CYCLES" \
            "SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_WAIT_ANY SQ_ACTIVE_INST_MISC" \
            "SQ_INSTS_VALU_MFMA_I8 SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_ANY SQ_INST_CYCLES_VMEM" ; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $ctrs --output-format csv -d $OUT/p$i -o run -- python3 ${PMC_CMD:-bench.py --steps 3 --warmup 1 --cpu-sample 0} > $OUT/p$i.log 2>&1 || echo "pass $i failed (rc $?)"
done
exit 0
