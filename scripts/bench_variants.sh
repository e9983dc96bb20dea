#!/bin/bash
# Quick bench of experiment builds: scripts/bench_variants.sh NAME... (lib/variants/libzd_NAME.so; "base" = lib/libzd.so)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for v in "$@"; do
  if [ "$v" = base ]; then lib=zstd-decompressor_amd/lib/libzd.so; else lib=zstd-decompressor_amd/lib/variants/libzd_$v.so; fi
  ZD_LIB_PATH=$lib ZD_CORPUS_CACHE=/tmp/zdc timeout -k 10 600 python bench.py --steps 3 --warmup 1 --unique-mib ${UMIB:-256} --replicas ${REPS:-4} --no-cpu-baseline --experiment > gpurun_out/var_$v.log 2>&1
  rc=$?
  echo "== $v rc=$rc"
  grep -o '"kernel_ms": {[^}]*}' gpurun_out/var_$v.log; grep -o '"verified_bit_exact": [a-z]*' gpurun_out/var_$v.log
  case $rc in 0) ;; *) echo "stop"; exit $rc;; esac
done
