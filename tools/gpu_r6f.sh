#!/bin/bash
# Round 6, session f: decode suite + the decode A/B (kernel-argument set, S = 1).
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_decode.py -m gpu -q -x -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/pytest_dec.log 2>&1; rc=$?; echo "pytest rc=$rc" >> gpurun_out/steps.log; [ $rc -le 1 ] || exit 3
timeout -k 10 300 python3 -u tools/decode_wall.py --knob rt_karg=1,0 --rounds 3 > gpurun_out/dec_ab.log 2>&1 || exit 3
echo "dec ok" >> gpurun_out/steps.log
