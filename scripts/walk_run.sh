#!/bin/bash
# Device header walk: its GPU test, then the C4 bench (reports device_walk_plan_ms beside host_plan_ms)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v -p no:cacheprovider --timeout 300 --timeout-method thread tests/test_gpu_walk.py > gpurun_out/walk_test.log 2>&1
rc=$?; echo "walk test rc=$rc"; tail -5 gpurun_out/walk_test.log
case $rc in 0|1) ;; *) exit $rc;; esac
ZD_PLAN_TIMES=1 timeout -k 10 600 python bench.py --steps 3 --warmup 1 --unique-mib 1024 --replicas 4 --no-cpu-baseline > gpurun_out/walk_bench.log 2>&1
rc=$?; echo "bench rc=$rc"; grep -o '"host_plan_ms": [^,]*, "host_plan_first_ms": [^,]*, "device_walk_plan_ms": [^,]*' gpurun_out/walk_bench.log; grep "zd device walk\|zd plan" gpurun_out/walk_bench.log | tail -8
exit $rc
