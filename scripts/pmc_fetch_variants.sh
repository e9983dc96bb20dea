#!/bin/bash
# FETCH_SIZE / WRITE_SIZE of each kernel for experiment builds (C4 at UMIB x REPS)
# usage: scripts/pmc_fetch_variants.sh NAME...   ("base" = lib/libzd.so)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp ZD_CORPUS_CACHE=/tmp/zdc
for v in "$@"; do
  if [ "$v" = base ]; then lib=zstd-decompressor_amd/lib/libzd.so; else lib=zstd-decompressor_amd/lib/variants/libzd_$v.so; fi
  for c in FETCH_SIZE WRITE_SIZE; do
    ZD_LIB_PATH=$lib timeout -k 10 300 rocprofv3 --kernel-trace --pmc $c -d gpurun_out/pmcv_${v}_$c -o run --output-format csv -- python bench.py --steps 1 --warmup 1 --unique-mib ${UMIB:-1024} --replicas ${REPS:-4} --no-cpu-baseline --no-verify --experiment > gpurun_out/pmcv_${v}_$c.log 2>&1
    rc=$?
    echo "== $v $c rc=$rc"
    case $rc in 0) ;; *) exit $rc;; esac
  done
  python scripts/pmc_summary.py gpurun_out/pmcv_${v}_* | grep -E "==|zd_k_execute|zd_k_sequences|zd_k_huffman"
done
