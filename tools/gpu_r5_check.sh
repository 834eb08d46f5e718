#!/bin/bash
# Round 5 check: the full GPU suite, flow-batch A/Bs (knobs flow_pipe,
# flow_fuse0), host root finding on the box's EPYC, and the u64 t=80 profile
# (kernel trace + SQ / FETCH passes).  STEPS selects.
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$ROOT/gpurun_out"
mkdir -p "$OUT"
cd "$ROOT"
export TMPDIR=/tmp
run() { local name=$1 to=$2; shift 2; echo "== $name" | tee -a "$OUT/steps.log"; timeout -k 10 "$to" "$@" > "$OUT/$name.log" 2>&1; local rc=$?; echo "== $name rc=$rc" | tee -a "$OUT/steps.log"; return $rc; }
for s in ${STEPS:-pytest abflows roots u64}; do
  case $s in
    pytest) run pytest 900 python3 -u -m pytest tests -m gpu -q -x -p no:cacheprovider -rA --timeout 300 --timeout-method thread || { [ $? -eq 1 ] || exit 3; } ;;
    smoke) run smoke 300 python3 -u -c "import __graft_entry__ as g; g.smoke()" || exit 3 ;;
    bench) run bench 600 python3 -u bench.py ${BENCH_ARGS:-} || exit 3 ;;
    abflows)
      run ab_pipe 600 python3 -u tools/ab_flows.py --knob flow_pipe --modes 1,0 --flows 16,10000,1000000 --rounds 4 || exit 3
      run ab_fuse0 600 python3 -u tools/ab_flows.py --knob flow_fuse0 --modes 1,0 --flows 16,10000,1000000 --rounds 4 || exit 3 ;;
    abflows1) run ab_flows 600 python3 -u tools/ab_flows.py --knob flow_sort --modes 2,1 --flows 16,10000,1000000 --rounds 4 || exit 3 ;;
    abocc) run ab_occ 600 python3 -u tools/ab_flows.py --knob flow_occ --modes 6,7 --flows 16,10000,1000000 --rounds 4 || exit 3 ;;
    pytestflows) run pytestflows 600 python3 -u -m pytest tests/test_flows.py tests/test_packets.py tests/test_gpu_variants.py -m gpu -q -x -p no:cacheprovider --timeout 300 --timeout-method thread -k "flow or knob or segment or packet" || { [ $? -eq 1 ] || exit 3; } ;;
    profflows) run profflows 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/profflows" -o run -- python3 "$ROOT/tools/ab_flows.py" --modes 2 --flows 16,10000,1000000 --rounds 3 || exit 3 ;;
    roots) run roots 300 python3 -u tools/bench_roots.py --d 8,16,32,64 --reps 400 || exit 3 ;;
    u64)
      run profu64 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/profu64" -o run -- python3 "$ROOT/tools/bench_configs.py" u64 --steps 10 || exit 3
      i=0
      for ctrs in "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVES GRBM_GUI_ACTIVE" \
                  "SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_WAVE_CYCLES SQ_BUSY_CYCLES" \
                  "SQ_INSTS_VALU_INT64 SQ_INSTS_VALU_INT32 SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_SALU" \
                  "FETCH_SIZE" ; do
        i=$((i+1))
        run pmcu64_$i 120 rocprofv3 --pmc $ctrs --output-format csv -d "$OUT/pmcu64_$i" -o run -- python3 "$ROOT/tools/bench_configs.py" u64 --steps 2 || exit 4
      done ;;
  esac
done
echo ALLDONE | tee -a "$OUT/steps.log"
