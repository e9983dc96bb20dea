#!/bin/bash
# Round-6 A/B 4: K4J rounds with each XCD's eighth swept as S regions
# (lib/variants/libzd_jsubS.so, ZD_J_SUB=S: a narrower sweep front, so more
# match sources lie behind it, already resolved in the same round) against
# the default (S = 1); and the hops per round (ZD_J_HOPS) at S = 1.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp ZD_CORPUS_CACHE=/tmp/zdc
V=zstd-decompressor_amd/lib/variants
ZD_LIB_PATH=$V/libzd_jsub8.so timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread \
  tests/test_large_frames.py "tests/test_fuzz.py::test_fuzz_block_parallel" "tests/test_gpu_parity.py::test_resources" \
  -m gpu > gpurun_out/ab4_pytest.log 2>&1; rc=$?
echo "pytest jsub8 rc=$rc"; tail -2 gpurun_out/ab4_pytest.log
[ $rc -eq 0 ] || exit $rc
run() {   # run NAME LIB WORKLOAD
  local out=gpurun_out/ab4_$1_$3.json
  if [ "$2" = default ]; then
    timeout -k 10 300 python bench.py --workload $3 --no-cpu-baseline --no-host-io > $out 2> ${out%.json}.err || exit 1
  else
    ZD_LIB_PATH=$V/libzd_$2.so timeout -k 10 300 python bench.py --workload $3 --no-cpu-baseline --no-host-io > $out 2> ${out%.json}.err || exit 1
  fi
  python -c "import json; d=json.load(open('$out')); print('$1 $3', d['value'], d['ms_per_step'], {k: v for k, v in d['kernel_ms'].items() if v > 0.01}, d['verified_bit_exact'])"
}
for i in 1 2; do
  run new$i default c3s; run jsub4_$i jsub4 c3s; run jsub8_$i jsub8 c3s; run jsub16_$i jsub16 c3s; run jsub32_$i jsub32 c3s
done
ZD_J_HOPS=4 run hops4 default c3s
ZD_J_HOPS=8 run hops8 default c3s
