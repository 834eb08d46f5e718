#!/bin/bash
# kernel traces of bench.cfg_flows with tools/ab/base.so and the in-tree library
set -u
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}"
mkdir -p gpurun_out
export TMPDIR=/tmp
for v in base new; do
  if [ $v = base ]; then export QK_LIB_PATH=$PWD/tools/ab/base.so; else unset QK_LIB_PATH; fi
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$v -o run -- python3 -u -c "
import bench
bench.cfg_flows(0)
" > gpurun_out/prof_$v.log 2>&1 || exit 3
done
