#!/bin/bash
# Round 6, session e: decode + comm suites (kernel-argument root-set scan,
# the RCCL pre-collective bound), the decode A/B, and the N = 8 bench
# rehearsed over the host channel on one GPU (8 ranks on one device).
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_decode.py tests/test_gpu_comm.py -m gpu -q -x -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/pytest_dec_comm.log 2>&1; rc=$?; echo "pytest rc=$rc" >> gpurun_out/steps.log; [ $rc -le 1 ] || exit 3
timeout -k 10 300 python3 -u tools/decode_wall.py --knob rt_karg=1,0 --rounds 3 > gpurun_out/dec_ab.log 2>&1 || exit 3
echo "dec ok" >> gpurun_out/steps.log
start=$(date +%s)
timeout -k 10 900 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 --master-port 29541 bench.py --gpus 8 > gpurun_out/dist8_host.log 2>&1; rc=$?
echo "dist8 rc=$rc wall_s=$(( $(date +%s) - start ))" >> gpurun_out/steps.log
