#!/bin/bash
# Round-6 GPU-box session: smoke, GPU parity suite, the bench line (with its
# N = 1 configs block), a process's first flow batch vs steady (16 / 1e6
# flows, one fresh process each), rocprofv3 kernel stats of the bench.
# Every step has its own time limit (tools/gpu_check.sh); results in gpurun_out/.
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$ROOT"
mkdir -p gpurun_out
STEPS="${R6_STEPS:-smoke pytest bench}" bash tools/gpu_check.sh || exit 3
for fl in ${COLD_FLOWS:-}; do
  echo "== cold $fl" >> gpurun_out/steps.log
  timeout -k 10 120 python3 -u tools/flows_cold.py --flows $fl >> gpurun_out/flows_cold.jsonl 2>> gpurun_out/flows_cold.err || exit 3
done
