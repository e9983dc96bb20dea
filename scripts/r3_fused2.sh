#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp ZD_CORPUS_CACHE=/tmp/zdc
ZD_FUSE=1 timeout -k 10 300 python bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-host-io --workload c3 > gpurun_out/r3fz2_c3.json 2> gpurun_out/r3fz2_c3.err; echo "c3 fuse rc=$?"; tail -5 gpurun_out/r3fz2_c3.err; head -c 400 gpurun_out/r3fz2_c3.json
