#!/bin/bash
# C3 (763 frames) bench of experiment builds: scripts/c3_variants.sh NAME... ("base" = lib/libzd.so)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for v in "$@"; do
  if [ "$v" = base ]; then lib=zstd-decompressor_amd/lib/libzd.so; else lib=zstd-decompressor_amd/lib/variants/libzd_$v.so; fi
  ZD_LIB_PATH=$lib ZD_CORPUS_CACHE=/tmp/zdc timeout -k 10 600 python bench.py --workload c3 --steps 5 --warmup 2 --no-cpu-baseline --experiment > gpurun_out/c3var_$v.log 2>&1
  rc=$?
  echo "== $v rc=$rc"
  grep -o '"value": [0-9.]*' gpurun_out/c3var_$v.log; grep -o '"kernel_ms": {[^}]*}' gpurun_out/c3var_$v.log; grep -o '"verified_bit_exact": [a-z]*' gpurun_out/c3var_$v.log
  case $rc in 0) ;; *) echo "stop"; exit $rc;; esac
done
