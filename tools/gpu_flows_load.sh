set -o pipefail
mkdir -p gpurun_out
for L in 4 2 8; do timeout -k 10 300 python -u tools/bench_configs.py flows --steps 6 --knob flow_load=$L > gpurun_out/flows_load$L.log 2>&1 || exit 1; done
