#!/bin/bash
# Round 5: flows parity on the hand-written grouping + kernel traces of the
# flow batches and of configs[2] (u64 t=80) + its SQ counter passes.
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$ROOT/gpurun_out"
mkdir -p "$OUT"
cd "$ROOT"
export TMPDIR=/tmp
run() { local name=$1 to=$2; shift 2; echo "== $name" | tee -a "$OUT/steps.log"; timeout -k 10 "$to" "$@" > "$OUT/$name.log" 2>&1; local rc=$?; echo "== $name rc=$rc" | tee -a "$OUT/steps.log"; return $rc; }
run pytest_flows 600 python3 -u -m pytest tests/test_flows.py tests/test_gpu_variants.py -m gpu -q -x -p no:cacheprovider --timeout 300 --timeout-method thread -k "flow or knob" || { [ $? -eq 1 ] || exit 3; }
run profflows 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/profflows" -o run -- python3 "$ROOT/tools/ab_flows.py" --modes 2 --flows 16,10000,1000000 --rounds 3 || exit 3
run profu64 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/profu64" -o run -- python3 "$ROOT/tools/bench_configs.py" u64 --steps 10 || exit 3
i=0
for ctrs in "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVES GRBM_GUI_ACTIVE" \
            "SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_WAVE_CYCLES SQ_BUSY_CYCLES" \
            "SQ_INSTS_VALU_INT64 SQ_INSTS_VALU_INT32 SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_SALU" \
            "FETCH_SIZE" ; do
  i=$((i+1))
  run pmcu64_$i 120 rocprofv3 --pmc $ctrs --output-format csv -d "$OUT/pmcu64_$i" -o run -- python3 "$ROOT/tools/bench_configs.py" u64 --steps 2 || exit 4
done
echo ALLDONE | tee -a "$OUT/steps.log"
