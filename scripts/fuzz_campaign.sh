#!/bin/bash
# Longer structure-aware fuzz campaigns of the GPU path against the oracle (tests/test_fuzz.py).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for seed in ${SEEDS:-1 2 3}; do
  ZD_FUZZ_SEED=$seed ZD_FUZZ_ITERS=${ITERS:-3000} ZD_FUZZ_PLAN_ITERS=${PLAN_ITERS:-300} timeout -k 10 600 python -m pytest tests/test_fuzz.py -q -s -p no:cacheprovider > gpurun_out/fuzz_$seed.log 2>&1
  rc=$?; echo "seed $seed rc=$rc $(tail -1 gpurun_out/fuzz_$seed.log)"
  [ $rc -eq 0 ] || exit $rc
done
