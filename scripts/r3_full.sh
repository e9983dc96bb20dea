#!/bin/bash
# the whole GPU suite as the driver runs it
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest -x -v -p no:cacheprovider --timeout 300 --timeout-method thread \
  tests -m gpu > gpurun_out/r3_full.log 2>&1
rc=$?; echo "tests rc=$rc"; grep -E "passed|failed|FAILED|Error" gpurun_out/r3_full.log | tail -8
exit $rc
