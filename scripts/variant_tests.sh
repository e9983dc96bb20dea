#!/bin/bash
# Runs one -m gpu test selection against experiment builds:
# scripts/variant_tests.sh "PYTEST -k EXPR" NAME...  (lib/variants/libzd_NAME.so; "base" = lib/libzd.so)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
sel=$1; shift
for v in "$@"; do
  if [ "$v" = base ]; then lib=zstd-decompressor_amd/lib/libzd.so; else lib=zstd-decompressor_amd/lib/variants/libzd_$v.so; fi
  ZD_LIB_PATH=$lib timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q -m gpu -p no:cacheprovider --timeout 120 --timeout-method thread -k "$sel" > gpurun_out/vt_$v.log 2>&1
  rc=$?
  echo "== $v rc=$rc $(tail -1 gpurun_out/vt_$v.log)"
  case $rc in 0|1) ;; *) echo "stop"; exit $rc;; esac
done
