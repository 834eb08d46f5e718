#!/bin/bash
# A/B of the per-flow batch (bench.cfg_flows, 1e6 flows) between the library
# at tools/ab/base.so and the in-tree one, alternating processes.
set -u
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}"
mkdir -p gpurun_out
for r in 1 2 3; do
  for v in base new; do
    if [ $v = base ]; then export QK_LIB_PATH=$PWD/tools/ab/base.so; else unset QK_LIB_PATH; fi
    timeout -k 10 200 python3 -u -c "
import json, bench
r = bench.cfg_flows(0)
print(json.dumps({'lib': '$v', 'steady': r['steady_ms_median'], 'min': r['steady_ms_min'], 'first': r['first_batch_ms'], 'ok': r['check']}))
" >> gpurun_out/flows_ab.log 2>&1 || exit 3
  done
done
