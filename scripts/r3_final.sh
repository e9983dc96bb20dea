#!/bin/bash
# round 3 final: the GPU suite as the driver runs it, smoke, then fuzz campaigns (outcome counts printed)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -v -p no:cacheprovider --timeout 300 --timeout-method thread \
  tests -m gpu > gpurun_out/r3_final_gpu.log 2>&1
rc=$?; echo "gpu suite rc=$rc"; grep -E "passed|failed|FAILED|Error" gpurun_out/r3_final_gpu.log | tail -5
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r3_final_smoke.log 2>&1; rc=$?; echo "smoke rc=$rc"; tail -1 gpurun_out/r3_final_smoke.log
[ $rc -eq 0 ] || exit $rc
for seed in ${SEEDS:-701 702 703}; do
  ZD_FUZZ_SEED=$seed ZD_FUZZ_ITERS=${ITERS:-10000} ZD_FUZZ_PLAN_ITERS=${PLAN_ITERS:-600} timeout -k 10 600 \
    python -u -m pytest tests/test_fuzz.py -v -s -p no:cacheprovider --timeout 550 --timeout-method thread > gpurun_out/fuzz_$seed.log 2>&1
  rc=$?; echo "fuzz seed $seed rc=$rc: $(grep -i 'outcome' gpurun_out/fuzz_$seed.log | tr '\n' ' ' | cut -c1-300) $(tail -1 gpurun_out/fuzz_$seed.log)"
  [ $rc -eq 0 ] || exit $rc
done
