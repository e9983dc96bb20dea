#!/bin/bash
# Quick bench under several environment settings: scripts/bench_env.sh "VAR=val ..." ...
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
i=0
for e in "$@"; do
  i=$((i+1))
  env $e timeout -k 10 600 python bench.py --steps 3 --warmup 1 --unique-mib ${UMIB:-256} --replicas ${REPS:-4} --no-cpu-baseline > gpurun_out/env_$i.log 2>&1
  rc=$?
  echo "== [$e] rc=$rc"
  grep -o '"value": [0-9.]*' gpurun_out/env_$i.log; grep -o '"kernel_ms": {[^}]*}' gpurun_out/env_$i.log; grep -o '"verified_bit_exact": [a-z]*' gpurun_out/env_$i.log
  case $rc in 0) ;; *) echo stop; exit $rc;; esac
done
