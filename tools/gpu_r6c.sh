#!/bin/bash
# Round 6, session c: (1) kernel trace of bench.py --comm (does a world-1
# in-place RCCL reduce enqueue kernels?), (2) the GPU suite without the
# RCCL abort test, (3) the decode call (overlapped root test), (4) the bench.
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
echo "== comm1" >> gpurun_out/steps.log
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/comm1 -o run -- python3 bench.py --comm --steps 3 --warmup 1 --ids-per-gpu 1e7 --configs 0 --cpu-sample 0 > gpurun_out/comm1.log 2>&1 || exit 3
echo "== pytest" >> gpurun_out/steps.log
timeout -k 10 900 python3 -u -m pytest tests -m gpu -q -x -p no:cacheprovider --timeout 300 --timeout-method thread -k "not pre_collective" > gpurun_out/pytest.log 2>&1; rc=$?; echo "pytest rc=$rc" >> gpurun_out/steps.log; [ $rc -le 1 ] || exit 3
echo "== dec" >> gpurun_out/steps.log
timeout -k 10 300 python3 -u tools/decode_wall.py > gpurun_out/dec.log 2>&1 || exit 3
echo "== bench" >> gpurun_out/steps.log
timeout -k 10 600 python3 -u bench.py > gpurun_out/bench.log 2>&1 || exit 3
echo "== done" >> gpurun_out/steps.log
