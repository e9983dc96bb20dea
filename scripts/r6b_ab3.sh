#!/bin/bash
# Round-6 A/B 3: K4J sweeps over round 1's pending list (default) against
# sweeps over every piece (lib/variants/libzd_jl0.so, ZD_J_LIST=0); K4J
# parity first (large single frames incl. 2.25 GiB, unconverged re-plans,
# block-parallel fuzz, forced K4J on the corpora).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp ZD_CORPUS_CACHE=/tmp/zdc
V=zstd-decompressor_amd/lib/variants
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_large_frames.py \
  "tests/test_fuzz.py::test_fuzz_block_parallel" "tests/test_gpu_parity.py::test_resources" \
  "tests/test_gpu_parity.py::test_synthetic_multi_block_frames" "tests/test_gpu_parity.py::test_one_round_plan" \
  -m gpu > gpurun_out/ab3_pytest.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -2 gpurun_out/ab3_pytest.log
[ $rc -eq 0 ] || exit $rc
run() {   # run NAME LIB WORKLOAD
  local out=gpurun_out/ab3_$1_$3.json
  if [ "$2" = default ]; then
    timeout -k 10 300 python bench.py --workload $3 --no-cpu-baseline --no-host-io > $out 2> ${out%.json}.err || exit 1
  else
    ZD_LIB_PATH=$V/libzd_$2.so timeout -k 10 300 python bench.py --workload $3 --no-cpu-baseline --no-host-io > $out 2> ${out%.json}.err || exit 1
  fi
  python -c "import json; d=json.load(open('$out')); print('$1 $3', d['value'], d['ms_per_step'], {k: v for k, v in d['kernel_ms'].items() if v > 0.01}, d['verified_bit_exact'])"
}
for i in 1 2 3; do
  run new$i default c3s; run jl0_$i jl0 c3s
done
