#!/bin/bash
# round 3: FSE tables built inside zd_k_fused (K1's sequence half off C3's critical path)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp ZD_CORPUS_CACHE=/tmp/zdc
timeout -k 10 300 python -u -m pytest -x -v -p no:cacheprovider --timeout 120 --timeout-method thread tests/test_gpu_parity.py -k "fused or mixed" > gpurun_out/r3fz4_t1.log 2>&1
rc=$?; echo "fused tests rc=$rc"; grep -E "passed|failed|FAILED|Error" gpurun_out/r3fz4_t1.log | tail -5; [ $rc = 0 ] || exit $rc
for i in 1 2; do
  timeout -k 10 300 python bench.py --workload c3 --steps 10 --warmup 3 --no-cpu-baseline --no-host-io > gpurun_out/r3fz4_c3_$i.json 2>gpurun_out/r3fz4_c3_$i.err; rc=$?
  echo "c3 rc=$rc"; [ $rc = 0 ] || exit $rc
  python -c "import json;d=json.load(open('gpurun_out/r3fz4_c3_$i.json'));print(d['value'],d['ms_per_step'],d.get('verified_bit_exact'))"
done
timeout -k 10 900 python -u -m pytest -x -v -p no:cacheprovider --timeout 300 --timeout-method thread tests -m gpu > gpurun_out/r3fz4_gpu.log 2>&1
rc=$?; echo "gpu suite rc=$rc"; grep -E "passed|failed|FAILED|Error" gpurun_out/r3fz4_gpu.log | tail -5; [ $rc = 0 ] || exit $rc
ZD_FUZZ_SEED=721 ZD_FUZZ_ITERS=3000 ZD_FUZZ_PLAN_ITERS=1500 timeout -k 10 600 \
  python -u -m pytest tests/test_fuzz.py -v -s -p no:cacheprovider --timeout 550 --timeout-method thread > gpurun_out/fuzz_721.log 2>&1
rc=$?; echo "fuzz rc=$rc: $(grep -i 'outcome' gpurun_out/fuzz_721.log | tr '\n' ' ' | cut -c1-400) $(tail -1 gpurun_out/fuzz_721.log)"
