set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_encode.py tests/test_gpu_variants.py -m gpu -x -q -k "u64 or grid_shape or misaligned" --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/pt_u64.log 2>&1 || exit 1
for sg in ${SGS:--1 20 12 8}; do
  timeout -k 10 120 python -u tools/bench_configs.py u64 --steps 5 --knob bsgs64_sg=$sg > gpurun_out/u64_sg$sg.log 2>&1 || exit 2
done
