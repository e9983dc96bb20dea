#!/bin/bash
# Round-end style run: default bench (JSON line -> gpurun_out/bench.json) and the
# rocprofv3 kernel-trace summary of the same command.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err; rc=$?
echo "bench rc=$rc"; tail -3 gpurun_out/bench.err; cat gpurun_out/bench.json
case $rc in 0) ;; *) exit $rc;; esac
timeout -k 10 900 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_full -o run --output-format csv -- python bench.py --no-cpu-baseline > gpurun_out/bench_prof.json 2> gpurun_out/bench_prof.err; rc=$?
echo "prof rc=$rc"; cat gpurun_out/prof_full/run_kernel_stats.csv | cut -c1-60,200-400 | head -8
exit $rc
