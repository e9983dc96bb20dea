#!/bin/bash
# Round-end style run on the GPU box: the default bench (JSON line ->
# gpurun_out/bench.json), the rocprofv3 kernel-trace summary of the same
# command, and the FETCH_SIZE / WRITE_SIZE passes for the traffic figures.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
export ZD_CORPUS_CACHE=/tmp/zdc
timeout -k 10 900 python bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err; rc=$?
echo "bench rc=$rc"; tail -3 gpurun_out/bench.err; cat gpurun_out/bench.json
[ $rc -eq 0 ] || exit $rc
timeout -k 10 900 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_full -o run --output-format csv -- python bench.py --no-cpu-baseline > gpurun_out/bench_prof.json 2> gpurun_out/bench_prof.err; rc=$?
echo "prof rc=$rc"
[ $rc -eq 0 ] || exit $rc
B="python bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-verify"
timeout -k 10 300 rocprofv3 --kernel-trace --pmc FETCH_SIZE -d gpurun_out/pmc_fetch -o run --output-format csv -- $B > gpurun_out/pmc_fetch.log 2>&1; rc=$?
echo "fetch rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --pmc WRITE_SIZE -d gpurun_out/pmc_write -o run --output-format csv -- $B > gpurun_out/pmc_write.log 2>&1; rc=$?
echo "write rc=$rc"; [ $rc -eq 0 ] || exit $rc
python scripts/pmc_traffic.py gpurun_out/pmc_fetch gpurun_out/pmc_write gpurun_out/traffic.json "${1:-}"
