#!/bin/bash
# Round-6 A/B 2 on one box (variants in lib/variants, ZD_LIB_PATH):
#   asm0      K3L without the one-op count sum and 64-bit funnel (ZD_K3L_ASM=0)
#   k3qd      K3Q with each window load issued after the next table read (ZD_K3Q_DEFER=1)
#   k3lprof*  K3L per-step ticks (ZD_K3L_PROF), with / without ZD_K3L_ASM
#   k3lraw    K3L with raw unformatted stores (timing only; it rejects, the
#             exact chain writes the records)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp ZD_CORPUS_CACHE=/tmp/zdc
V=zstd-decompressor_amd/lib/variants
timeout -k 10 500 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_large_frames.py \
  tests/test_frame_iterator.py "tests/test_gpu_parity.py::test_fused_plans" "tests/test_fuzz.py::test_fuzz_block_parallel" \
  "tests/test_gpu_parity.py::test_one_lane_k3_chain" "tests/test_gpu_parity.py::test_synthetic_multi_block_frames" \
  -m gpu > gpurun_out/ab2_pytest.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -2 gpurun_out/ab2_pytest.log
[ $rc -eq 0 ] || exit $rc
ZD_LIB_PATH=$V/libzd_k3qd.so timeout -k 10 500 python -u -m pytest -x -q --timeout 200 --timeout-method thread \
  "tests/test_gpu_parity.py::test_synthetic_single_block_frames" "tests/test_gpu_parity.py::test_corrupted_inputs" \
  "tests/test_gpu_parity.py::test_resources" "tests/test_fuzz.py::test_fuzz_structure_aware" \
  -m gpu > gpurun_out/ab2_pytest_k3qd.log 2>&1; rc=$?
echo "pytest k3qd rc=$rc"; tail -2 gpurun_out/ab2_pytest_k3qd.log
[ $rc -eq 0 ] || exit $rc
run() {   # run NAME LIB WORKLOAD [extra]
  local out=gpurun_out/ab2_$1_$3.json
  if [ "$2" = default ]; then
    timeout -k 10 300 python bench.py --workload $3 --no-cpu-baseline --no-host-io ${4:-} > $out 2> ${out%.json}.err || exit 1
  else
    ZD_LIB_PATH=$V/libzd_$2.so timeout -k 10 300 python bench.py --workload $3 --no-cpu-baseline --no-host-io ${4:-} > $out 2> ${out%.json}.err || exit 1
  fi
  python -c "import json; d=json.load(open('$out')); print('$1 $3', d['value'], d['ms_per_step'], {k: v for k, v in d['kernel_ms'].items() if v > 0.01}, d['verified_bit_exact'])"
}
for i in 1 2; do
  run new$i default c3s; run asm0_$i asm0 c3s
  run new$i default c3; run asm0_$i asm0 c3
done
for i in 1 2; do
  run new$i default c4; run k3qd_$i k3qd c4
done
for v in k3lprof k3lprofasm0 k3lraw; do
  ZD_LIB_PATH=$V/libzd_$v.so timeout -k 10 200 python bench.py --workload c3s --no-cpu-baseline --no-host-io --no-verify --steps 1 --warmup 1 \
    > gpurun_out/ab2_$v.json 2> gpurun_out/ab2_$v.err || exit 1
  echo "== $v"; cat gpurun_out/ab2_$v.err gpurun_out/ab2_$v.json | grep -a "K3L block" | head -4
done
timeout -k 10 300 python scripts/time_frame_iterator.py gpurun_out/ab2_frame_iterator.json || exit 1
