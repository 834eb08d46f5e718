#!/bin/bash
# Round 6 closing pass on one GPU box: smoke, the GPU suite, the bench line
# (with its configs block), a kernel trace + stats and a FETCH_SIZE pass of
# the same bench command (tools/r6_roofline.py), and the two-rank rehearsal.
# Every GPU step has its own time limit (tools/gpu_check.sh).
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$ROOT"
mkdir -p gpurun_out
STEPS="${FINAL_STEPS:-smoke pytest bench}" bash tools/gpu_check.sh || exit 3
export TMPDIR=/tmp
if [ -z "${SKIP_PROF:-}" ]; then
  echo "== prof" >> gpurun_out/steps.log
  timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o run -- python3 bench.py --steps 20 --warmup 1 --cpu-sample 0 > gpurun_out/prof.log 2>&1 || exit 3
  echo "== pmc" >> gpurun_out/steps.log
  timeout -k 10 600 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmc -o run -- python3 bench.py --steps 3 --warmup 1 --cpu-sample 0 > gpurun_out/pmc.log 2>&1 || exit 3
  python3 tools/r6_roofline.py gpurun_out > gpurun_out/roofline.json 2>> gpurun_out/steps.log
fi
if [ -z "${SKIP_DIST:-}" ]; then
  echo "== dist2" >> gpurun_out/steps.log
  timeout -k 10 600 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29535 bench.py --gpus 2 --steps 3 --warmup 1 --cpu-sample 0 > gpurun_out/dist2.log 2>&1 || exit 3
fi
echo "== done" >> gpurun_out/steps.log
