#!/bin/bash
# Copy a gpurun_out/ session into profiles/r06/<name>/ (logs, JSON lines,
# rocprofv3 stats; full traces over 2 MB are left out) and clear gpurun_out/.
set -eu
name=$1
dst=profiles/r06/$name
mkdir -p "$dst"
( cd gpurun_out && find . -type f ! -name ".last_call.json" -size -2M -print0 | tar --null -cf - -T - ) | tar -xf - -C "$dst"
rm -rf gpurun_out/*
echo "saved to $dst"; find "$dst" -type f | head -30
