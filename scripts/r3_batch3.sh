#!/bin/bash
# round 3 batch 3: packed K4 scan + K4J for few-frame plans -- parity, C4 4 GiB / 1 GiB vs r3b, few-frames timing
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp ZD_CORPUS_CACHE=/tmp/zdc
timeout -k 10 600 python -u -m pytest -x -v -p no:cacheprovider --timeout 300 --timeout-method thread \
  tests/test_gpu_parity.py tests/test_large_frames.py tests/test_k4f.py tests/test_resource_digests.py -m gpu > gpurun_out/r3_t3.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -4 gpurun_out/r3_t3.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python scripts/time_small.py > gpurun_out/r3_small.json 2> gpurun_out/r3_small.err; echo "small rc=$?"; cat gpurun_out/r3_small.err | grep -v amdgpu.ids
UMIB=1024 REPS=4 bash scripts/bench_variants.sh r3b base r3b base || exit $?
UMIB=256 REPS=4 bash scripts/bench_variants.sh r3b base || exit $?
timeout -k 10 60 rocprofv3 -L > gpurun_out/r3_counters.txt 2>&1; echo "list rc=$?"; grep -i -E "RDREQ|EA0_RD|TCC_REQ|TCC_READ" gpurun_out/r3_counters.txt | head -30
