#!/bin/bash
# A/B of the streaming executors on C4 (4 GiB): ZD_K4P=0 (K4) vs 1 (K4P)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out
export ZD_CORPUS_CACHE=/tmp/zdc
for v in ${K4P_LIST:-0 1}; do
  ZD_K4P=$v timeout -k 10 600 python bench.py --steps 3 --warmup 1 --unique-mib ${UMIB:-1024} --replicas ${REPS:-4} --no-cpu-baseline --experiment > gpurun_out/k4p_$v.log 2>&1
  rc=$?; echo "K4P=$v rc=$rc $(grep -o '"zd_k_execute": [0-9.]*' gpurun_out/k4p_$v.log) $(grep -o '"verified_bit_exact": [a-z]*' gpurun_out/k4p_$v.log)"
  [ $rc -eq 0 ] || exit $rc
done
