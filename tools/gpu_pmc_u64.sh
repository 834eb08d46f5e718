# PMC passes over the u64 t=80 encode (tools/bench_configs.py u64), one counter group per run.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/pmc_u64
mkdir -p $OUT
i=0
for ctrs in "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVES GRBM_GUI_ACTIVE" \
            "SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_WAVE_CYCLES SQ_BUSY_CYCLES" \
            "SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_WAIT_ANY SQ_INST_CYCLES_SALU" ; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $ctrs --output-format csv -d $OUT/p$i -o run -- python3 tools/bench_configs.py u64 --steps 2 > $OUT/p$i.log 2>&1 || exit $i
done
