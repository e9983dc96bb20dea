#!/bin/bash
# round 3: FSE tables built by the K4 waves of zd_k_fused (64 lanes a table)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp ZD_CORPUS_CACHE=/tmp/zdc
timeout -k 10 300 python -u -m pytest -x -v -p no:cacheprovider --timeout 120 --timeout-method thread tests/test_gpu_parity.py -k "fused or mixed" > gpurun_out/r3fz5_t1.log 2>&1
rc=$?; echo "fused tests rc=$rc"; grep -E "passed|failed|FAILED|Error" gpurun_out/r3fz5_t1.log | tail -5; [ $rc = 0 ] || exit $rc
for i in 1 2; do
  timeout -k 10 300 python bench.py --workload c3 --steps 10 --warmup 3 --no-cpu-baseline --no-host-io > gpurun_out/r3fz5_c3_$i.json 2>gpurun_out/r3fz5_c3_$i.err; rc=$?
  echo "c3 rc=$rc"; [ $rc = 0 ] || exit $rc
  python -c "import json;d=json.load(open('gpurun_out/r3fz5_c3_$i.json'));print(d['value'],d['ms_per_step'],d.get('verified_bit_exact'))"
done
ZD_LIB_PATH=zstd-decompressor_amd/lib/variants/libzd_fztrace.so timeout -k 10 300 python scripts/fztrace.py > gpurun_out/fztrace5.log 2>&1; rc=$?; grep -v amdgpu.ids gpurun_out/fztrace5.log | tail -3; [ $rc = 0 ] || exit $rc
ZD_FUZZ_SEED=732 ZD_FUZZ_ITERS=500 ZD_FUZZ_PLAN_ITERS=1500 timeout -k 10 600 \
  python -u -m pytest tests/test_fuzz.py -v -s -p no:cacheprovider --timeout 550 --timeout-method thread > gpurun_out/fuzz_732.log 2>&1
rc=$?; echo "fuzz rc=$rc: $(grep -i 'outcome' gpurun_out/fuzz_732.log | tr '\n' ' ' | cut -c1-400) $(tail -1 gpurun_out/fuzz_732.log)"
