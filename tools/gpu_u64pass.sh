#!/bin/bash
# u64 t > 80: multi-pass BSGS parity tests, then sweep64 default vs chain
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_encode.py -m gpu -x -q -k "u64" --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/pt_u64pass.log 2>&1 || exit 1
timeout -k 10 300 python -u tools/bench_configs.py sweep64 --steps 6 > gpurun_out/sweep64_pass.log 2>&1 || exit 2

timeout -k 10 300 python -u tools/bench_configs.py u64 --steps 10 > gpurun_out/u64_t80.log 2>&1 || exit 4
