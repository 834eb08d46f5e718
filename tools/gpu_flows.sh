#!/bin/bash
# per-flow batches: GPU parity tests, then the flows bench and a kernel trace
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_flows.py tests/test_gpu_encode.py -k "flows or segment or seg or grid_shape" -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/pt_flows.log 2>&1 || exit 1
timeout -k 10 300 python -u tools/bench_configs.py flows --steps 6 > gpurun_out/flows.log 2>&1 || exit 2
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/proflows -o run -- python3 tools/bench_configs.py flows --steps 4 > gpurun_out/proflows.log 2>&1 || exit 3
