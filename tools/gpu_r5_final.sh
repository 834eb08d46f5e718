#!/bin/bash
# Round-5 closing measurement on one GPU box: smoke, the GPU parity suite,
# the bench line, its rocprofv3 kernel trace and FETCH_SIZE pass, the
# secondary configs (+ their kernel stats), the host root finding, the
# two-rank rehearsal of the N>1 bench, and the roots A/B on the host CPU.
# Every step runs under its own time limit (tools/gpu_check.sh); results in
# gpurun_out/.
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$ROOT"
mkdir -p gpurun_out
timeout -k 10 200 ./tools/prof_roots 32 200 > gpurun_out/prof_roots.txt 2>&1 || exit 3
CONFIGS_ARGS="u64 decode decode64 flows packets" \
STEPS="smoke pytest bench prof pmc configs roots dist2full profcfg pmccfg proflows" bash tools/gpu_check.sh
