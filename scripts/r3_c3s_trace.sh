#!/bin/bash
# round 3: kernel trace of the single-frame C3 (K4J) pipeline
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/r3_c3s_trace -o run --output-format csv -- python bench.py --workload c3s --steps 2 --warmup 1 --no-cpu-baseline --no-host-io > gpurun_out/r3_c3s_trace.log 2>&1; echo "trace rc=$?"
