#!/bin/bash
# Round 6, session d: decode A/B (overlapped root test on / off) and its
# trace; the RCCL pre-collective bounded-wait test.
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python3 -u tools/decode_wall.py --knob rt_overlap=1,0 --rounds 3 > gpurun_out/dec_ab.log 2>&1 || exit 3
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --hip-runtime-trace --output-format csv -d gpurun_out/dec -o run -- python3 tools/decode_wall.py --bits 32 --reps 10 --knob rt_overlap=1,0 > gpurun_out/dec_trace.log 2>&1 || exit 3
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_comm.py -m gpu -q -x -p no:cacheprovider --timeout 120 --timeout-method thread -k "pre_collective" > gpurun_out/pytest_pre.log 2>&1; echo "pre rc=$?" >> gpurun_out/steps.log
