#!/bin/bash
# Round-6 A/B 15: FwBitsW (the wave-parallel table parse) with 32-bit bookkeeping (ZD_FWW32,
# default) against 64-bit (lib/variants/libzd_w64.so), on top of the lane-mask build;
# c3s (zd_k_tables_seqw ahead of the chains) and C3 (zd_k_fused).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp ZD_CORPUS_CACHE=/tmp/zdc
V=zstd-decompressor_amd/lib/variants
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread \
  "tests/test_gpu_parity.py::test_fused_plans" "tests/test_gpu_parity.py::test_fused_table_builds" \
  "tests/test_gpu_parity.py::test_k1_large_tables" "tests/test_gpu_parity.py::test_synthetic_single_block_frames" \
  "tests/test_gpu_parity.py::test_corrupted_inputs" "tests/test_gpu_parity.py::test_corrupted_inputs_forked_plan" \
  tests/test_fuzz.py tests/test_large_frames.py -m gpu > gpurun_out/ab15_pytest.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -2 gpurun_out/ab15_pytest.log
[ $rc -eq 0 ] || exit $rc
run() {   # run NAME LIB WORKLOAD
  local out=gpurun_out/ab15_$1_$3.json
  if [ "$2" = default ]; then
    timeout -k 10 300 python bench.py --workload $3 --no-cpu-baseline --no-host-io > $out 2> ${out%.json}.err || exit 1
  else
    ZD_LIB_PATH=$V/libzd_$2.so timeout -k 10 300 python bench.py --workload $3 --no-cpu-baseline --no-host-io > $out 2> ${out%.json}.err || exit 1
  fi
  python -c "import json; d=json.load(open('$out')); print('$1 $3', d['value'], d['ms_per_step'], d['roofline']['kernel_ms'], d['kernel_ms'].get('zd_k_tables'), d['verified_bit_exact'])"
}
for i in 1 2 3; do
  run new$i default c3s; run w64_$i w64 c3s
  run new$i default c3; run w64_$i w64 c3
done
