#!/bin/bash
# round 3: K2 compact LUT vs the 4 KiB LUT on C4 10 GiB (8 rounds of K2 blocks before, 5 after)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp ZD_CORPUS_CACHE=/tmp/zdc
UMIB=1024 REPS=10 bash scripts/bench_variants.sh base k2old k2c16 base k2old k2c16
