#!/bin/bash
# round 3 batch 4: capacity re-plans in zd_plan_decompress -- parity + the seed-601 fuzz campaign (OOD count)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v -p no:cacheprovider --timeout 300 --timeout-method thread \
  tests/test_gpu_parity.py tests/test_host_io.py tests/test_large_frames.py -m gpu > gpurun_out/r3_t4.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -4 gpurun_out/r3_t4.log
[ $rc -eq 0 ] || exit $rc
rm -rf gpurun_out/ood2
ZD_FUZZ_ITERS=3000 ZD_FUZZ_PLAN_ITERS=300 ZD_FUZZ_SEED=601 ZD_FUZZ_DUMP=gpurun_out/ood2 timeout -k 10 700 python -u -m pytest -x -v -s -p no:cacheprovider --timeout 600 --timeout-method thread tests/test_fuzz.py > gpurun_out/r3_fuzz601b.log 2>&1; echo "fuzz rc=$?"; grep "outcome\|FAIL\|Error" gpurun_out/r3_fuzz601b.log | head
