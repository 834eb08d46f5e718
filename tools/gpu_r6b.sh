#!/bin/bash
# Round 6, session b: (1) does a world-1 RCCL reduce launch kernels (kernel
# trace of bench.py --comm), (2) the decode call's kernel / copy / HIP-API
# trace, (3) the bench line with the core-cycle CPU baseline.
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/comm1 -o run -- python3 bench.py --comm --steps 3 --warmup 1 --ids-per-gpu 1e7 --configs 0 --cpu-sample 0 > gpurun_out/comm1.log 2>&1 || exit 3
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --hip-runtime-trace --output-format csv -d gpurun_out/dec -o run -- python3 tools/decode_wall.py --reps 20 > gpurun_out/dec.log 2>&1 || exit 3
timeout -k 10 600 python3 -u bench.py > gpurun_out/bench.log 2>&1 || exit 3
