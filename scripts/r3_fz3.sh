#!/bin/bash
# round 3: zd_k_fused layout variants on C3 (chain-wave priority, publish interval, chain wave alone on its SIMD)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp ZD_CORPUS_CACHE=/tmp/zdc
ZD_LIB_PATH=zstd-decompressor_amd/lib/variants/libzd_solo6.so timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py -k fused > gpurun_out/r3fz3_test.log 2>&1; rc=$?; tail -3 gpurun_out/r3fz3_test.log; [ $rc = 0 ] || exit $rc
for v in base pr3 pub32 solo6 solo6pr3 base pr3 pub32 solo6 solo6pr3; do
  if [ $v = base ]; then lib=zstd-decompressor_amd/lib/libzd.so; else lib=zstd-decompressor_amd/lib/variants/libzd_$v.so; fi
  ZD_LIB_PATH=$lib timeout -k 10 300 python bench.py --workload c3 --steps 10 --warmup 3 --no-cpu-baseline --no-host-io > gpurun_out/r3fz3_$v.json 2>gpurun_out/r3fz3_$v.err; rc=$?
  echo "c3 $v rc=$rc"; [ $rc = 0 ] || exit $rc
  python -c "import json;d=json.load(open('gpurun_out/r3fz3_$v.json'));print(d['value'],d['ms_per_step'],d.get('verified_bit_exact'))"
done
