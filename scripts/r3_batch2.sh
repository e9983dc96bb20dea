#!/bin/bash
# round 3 batch 2: 4 GiB C4 (r3a vs current), FETCH_SIZE calibration, a fuzz
# campaign keeping out-of-domain inputs, and the default bench line
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp ZD_CORPUS_CACHE=/tmp/zdc
UMIB=1024 REPS=4 bash scripts/bench_variants.sh r3a base || exit $?
timeout -k 10 120 rocprofv3 --kernel-trace --pmc FETCH_SIZE -d gpurun_out/r3_calib -o run --output-format csv -- tools/fetch_calib > gpurun_out/r3_calib.log 2>&1; echo "calib rc=$?"
ZD_FUZZ_ITERS=3000 ZD_FUZZ_PLAN_ITERS=300 ZD_FUZZ_SEED=601 ZD_FUZZ_DUMP=gpurun_out/ood timeout -k 10 600 python -u -m pytest -x -v -s -p no:cacheprovider --timeout 500 --timeout-method thread tests/test_fuzz.py > gpurun_out/r3_fuzz601.log 2>&1; echo "fuzz rc=$?"; grep "outcome" gpurun_out/r3_fuzz601.log
timeout -k 10 900 python bench.py > gpurun_out/r3_bench.json 2> gpurun_out/r3_bench.err; echo "bench rc=$?"; tail -3 gpurun_out/r3_bench.err; cat gpurun_out/r3_bench.json
