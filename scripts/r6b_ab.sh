#!/bin/bash
# Round-6 A/B on one box (timing-only and macro variants in lib/variants,
# selected with ZD_LIB_PATH; the default build is lib/libzd.so):
#   js0        the round-5 scatter (ZD_JS_STAGE=0: literal bytes one HBM load
#              each, a division per overlapping match byte)
#   sh0        K3L pair formatting where the compiler puts it (ZD_K3L_SHADOW=0)
#   k3lprof*   K3L per-step ticks (ZD_K3L_PROF), with / without the shadow
#   k3lraw     K3L with raw unformatted stores (timing only: it rejects, the
#              exact chain writes the records)
# Parity of the default build on the K4J and K3L paths first.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp ZD_CORPUS_CACHE=/tmp/zdc
V=zstd-decompressor_amd/lib/variants
timeout -k 10 500 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_large_frames.py \
  tests/test_fuzz.py tests/test_frame_iterator.py "tests/test_gpu_parity.py::test_fused_plans" \
  "tests/test_gpu_parity.py::test_one_lane_k3_chain" "tests/test_gpu_parity.py::test_synthetic_multi_block_frames" \
  -m gpu > gpurun_out/ab_pytest.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -2 gpurun_out/ab_pytest.log
[ $rc -eq 0 ] || exit $rc
run() {   # run NAME LIB WORKLOAD
  local out=gpurun_out/ab_$1_$3.json
  if [ "$2" = default ]; then
    timeout -k 10 200 python bench.py --workload $3 --no-cpu-baseline --no-host-io > $out 2> ${out%.json}.err || exit 1
  else
    ZD_LIB_PATH=$V/libzd_$2.so timeout -k 10 200 python bench.py --workload $3 --no-cpu-baseline --no-host-io > $out 2> ${out%.json}.err || exit 1
  fi
  python -c "import json; d=json.load(open('$out')); print('$1 $3', d['value'], d['ms_per_step'], {k: v for k, v in d['kernel_ms'].items() if v > 0.01}, d['verified_bit_exact'])"
}
for i in 1 2; do
  run new$i default c3s; run js0_$i js0 c3s; run sh0_$i sh0 c3s
  run new$i default c3; run sh0_$i sh0 c3
done
for v in k3lprof k3lprofsh0 k3lraw; do
  ZD_LIB_PATH=$V/libzd_$v.so timeout -k 10 200 python bench.py --workload c3s --no-cpu-baseline --no-host-io --no-verify --steps 1 --warmup 0 \
    > gpurun_out/ab_$v.json 2> gpurun_out/ab_$v.err || exit 1
  echo "== $v"; cat gpurun_out/ab_$v.err gpurun_out/ab_$v.json | grep -a "K3L block" | head -4
done
timeout -k 10 300 python scripts/time_frame_iterator.py gpurun_out/ab_frame_iterator.json || exit 1
