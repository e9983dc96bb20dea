#!/bin/bash
# Few-frames thresholds: K2 | K3 fork and K4F at 8192 and 16384 frames (1 / 2 GiB of C4 frames).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp ZD_CORPUS_CACHE=/tmp/zdc
for reps in 4 8; do
  for v in "ZD_FORK=0 ZD_K4F=0" "ZD_FORK=1 ZD_K4F=0" "ZD_FORK=0 ZD_K4F=1" "ZD_FORK=1 ZD_K4F=1"; do
    env $v timeout -k 10 300 python bench.py --steps 3 --warmup 1 --unique-mib 256 --replicas $reps --no-cpu-baseline > gpurun_out/thr.json 2> gpurun_out/thr.err || exit $?
    echo "reps=$reps $v $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/thr.json) $(grep -o '"verified_bit_exact": [a-z]*' gpurun_out/thr.json)"
  done
done
