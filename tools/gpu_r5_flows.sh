#!/bin/bash
# Round 5: flows parity + per-call kernel trace of the flow batches.
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$ROOT/gpurun_out"
mkdir -p "$OUT"
cd "$ROOT"
export TMPDIR=/tmp
run() { local name=$1 to=$2; shift 2; echo "== $name" | tee -a "$OUT/steps.log"; timeout -k 10 "$to" "$@" > "$OUT/$name.log" 2>&1; local rc=$?; echo "== $name rc=$rc" | tee -a "$OUT/steps.log"; return $rc; }
run pytest_flows 600 python3 -u -m pytest tests/test_flows.py tests/test_gpu_variants.py tests/test_packets.py -m gpu -q -x -p no:cacheprovider --timeout 300 --timeout-method thread -k "flow or knob or segment or packet" || { [ $? -eq 1 ] || exit 3; }
run abflows 600 python3 -u tools/ab_flows.py --modes ${FLOW_MODES:-2,1} --flows 16,10000,1000000 --rounds 4 || exit 3
run profflows 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/profflows" -o run -- python3 "$ROOT/tools/ab_flows.py" --modes 2 --flows 16,10000,1000000 --rounds 3 || exit 3
echo ALLDONE | tee -a "$OUT/steps.log"
