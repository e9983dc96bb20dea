#!/bin/bash
# round 3: K1 table builds without LDS reloads (spread count in a register, restrict LUT/table pointers)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp ZD_CORPUS_CACHE=/tmp/zdc
timeout -k 10 900 python -u -m pytest -x -v -p no:cacheprovider --timeout 300 --timeout-method thread \
  tests/test_gpu_parity.py tests/test_fuzz.py -m gpu > gpurun_out/r3k1_t.log 2>&1
rc=$?; echo "tests rc=$rc"; grep -E "passed|failed|FAILED|Error" gpurun_out/r3k1_t.log | tail -8
[ $rc -eq 0 ] || exit $rc
bash scripts/bench_variants.sh base k1old base k1old
for v in base k1old; do
  if [ $v = base ]; then lib=zstd-decompressor_amd/lib/libzd.so; else lib=zstd-decompressor_amd/lib/variants/libzd_$v.so; fi
  ZD_LIB_PATH=$lib timeout -k 10 300 python bench.py --workload c3 --steps 5 --warmup 2 --no-cpu-baseline --no-host-io > gpurun_out/r3k1_c3_$v.json 2>/dev/null; echo "c3 $v rc=$?"
  python -c "import json;d=json.load(open('gpurun_out/r3k1_c3_$v.json'));print(d['ms_per_step'],d['kernel_ms'])"
done
