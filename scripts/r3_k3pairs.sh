#!/bin/bash
# round 3: record pairs (K3 without cross-lane packing) -- parity, then C4 4 GiB vs the r3a build
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp ZD_CORPUS_CACHE=/tmp/zdc
timeout -k 10 300 python -u -m pytest -x -v -p no:cacheprovider --timeout 100 --timeout-method thread \
  tests/test_gpu_parity.py::test_resources tests/test_gpu_parity.py::test_one_lane_k3_chain > gpurun_out/r3_t0.log 2>&1
rc=$?; echo "quick tests rc=$rc"; tail -5 gpurun_out/r3_t0.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python -u -m pytest -x -v -p no:cacheprovider --timeout 300 --timeout-method thread \
  tests/test_gpu_parity.py tests/test_host_io.py tests/test_gpu_walk.py tests/test_shard.py -m gpu > gpurun_out/r3_t1.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -15 gpurun_out/r3_t1.log
case $rc in 0|1) ;; *) exit $rc;; esac
bash scripts/bench_variants.sh r3a base r3a base
