#!/bin/bash
# C3 (763 frames, the latency-bound regime): streaming K4 (forced) vs the
# frame-in-LDS executor K4F, then the default bench line.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp ZD_CORPUS_CACHE=/tmp/zdc
ZD_K4F=0 timeout -k 10 300 python bench.py --workload c3 --no-cpu-baseline > gpurun_out/c3_k4.json 2> gpurun_out/c3_k4.err || exit $?
cat gpurun_out/c3_k4.json
ZD_K4F=1 timeout -k 10 300 python bench.py --workload c3 --no-cpu-baseline > gpurun_out/c3_k4f.json 2> gpurun_out/c3_k4f.err || exit $?
cat gpurun_out/c3_k4f.json
[ "${1:-}" = "full" ] || exit 0
timeout -k 10 900 python bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err || exit $?
cat gpurun_out/bench.json
