#!/bin/bash
# K3/K4 overlap across frame halves (ZD_OVERLAP=1) against the serial pipeline, C4 1 GiB x10.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for ov in 0 1 0 1; do
  ZD_OVERLAP=$ov ZD_CORPUS_CACHE=/tmp/zdc timeout -k 10 600 python bench.py --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/ov_$ov.log 2>&1 || { echo "rc=$? overlap=$ov"; tail -5 gpurun_out/ov_$ov.log; exit 1; }
  echo "overlap=$ov $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/ov_$ov.log) $(grep -o '"verified_bit_exact": [a-z]*' gpurun_out/ov_$ov.log)"
done
