#!/bin/bash
# round 3 re-entry: GPU suite, then the C4 bench line and its rocprofv3 kernel stats
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
export ZD_CORPUS_CACHE=/tmp/zdc
timeout -k 10 1000 python -u -m pytest -x -v -p no:cacheprovider --timeout 300 --timeout-method thread \
  tests -m gpu > gpurun_out/r3c_full.log 2>&1
rc=$?; echo "tests rc=$rc"; grep -E "passed|failed|FAILED|Error" gpurun_out/r3c_full.log | tail -8
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python bench.py > gpurun_out/r3c_c4.json 2> gpurun_out/r3c_c4.err; rc=$?
echo "bench rc=$rc"; cat gpurun_out/r3c_c4.json; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/r3c_prof_c4 -o run --output-format csv -- python bench.py --no-cpu-baseline > gpurun_out/r3c_prof.log 2>&1; echo "prof rc=$?"
