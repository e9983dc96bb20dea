#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
ZD_LIB_PATH=zstd-decompressor_amd/lib/variants/libzd_k1prof.so timeout -k 10 300 python scripts/k1prof.py > gpurun_out/r3_k1prof.log 2>&1; echo "rc=$?"; cat gpurun_out/r3_k1prof.log | tail -5
