#!/bin/bash
# round 3: K2 compact two-level LDS LUT (P: 10 bits + the 11-bit head) -- parity, then C4 1 GiB vs the 4 KiB LUT
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp ZD_CORPUS_CACHE=/tmp/zdc
timeout -k 10 900 python -u -m pytest -x -v -p no:cacheprovider --timeout 300 --timeout-method thread \
  tests/test_gpu_parity.py tests/test_fuzz.py tests/test_resource_digests.py -m gpu > gpurun_out/r3k2_t.log 2>&1
rc=$?; echo "tests rc=$rc"; grep -E "passed|failed|FAILED|Error" gpurun_out/r3k2_t.log | tail -8
[ $rc -eq 0 ] || exit $rc
bash scripts/bench_variants.sh base k2old k2c16 k2c4 base k2old k2c16 k2c4
