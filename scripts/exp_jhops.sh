#!/bin/bash
# K4J hops per round (ZD_J_HOPS) on the single-frame C3 (c3s) workload.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out
for h in ${HOPS:-1 2 4 8}; do
  ZD_J_HOPS=$h timeout -k 10 300 python bench.py --workload c3s --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/jhops_$h.log 2>&1 || exit $?
  echo "hops=$h $(grep '^{' gpurun_out/jhops_$h.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["kernel_ms"])')"
done
