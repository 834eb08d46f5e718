#!/bin/bash
# decode: GPU parity tests (root test, receiver, comm), then the configs[4] rows
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_decode.py tests/test_receiver.py tests/test_gpu_comm.py -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/pt_decode.log 2>&1 || exit 1
timeout -k 10 300 python -u tools/bench_configs.py decode decode64 --steps 10 > gpurun_out/decode.log 2>&1 || exit 2
