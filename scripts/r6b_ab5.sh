#!/bin/bash
# Round-6 A/B 5: K4J rounds with the chip in ZD_J_XREG = 4 / 2 / 1 regions (each swept by the
# workgroups of 2 / 4 / 8 XCDs; lib/variants/libzd_xregN.so) against one region an XCD.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp ZD_CORPUS_CACHE=/tmp/zdc
V=zstd-decompressor_amd/lib/variants
ZD_LIB_PATH=$V/libzd_xreg1.so timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread \
  tests/test_large_frames.py "tests/test_fuzz.py::test_fuzz_block_parallel" "tests/test_gpu_parity.py::test_resources" \
  -m gpu > gpurun_out/ab5_pytest.log 2>&1; rc=$?
echo "pytest xreg1 rc=$rc"; tail -2 gpurun_out/ab5_pytest.log
[ $rc -eq 0 ] || exit $rc
run() {   # run NAME LIB WORKLOAD
  local out=gpurun_out/ab5_$1_$3.json
  if [ "$2" = default ]; then
    timeout -k 10 300 python bench.py --workload $3 --no-cpu-baseline --no-host-io > $out 2> ${out%.json}.err || exit 1
  else
    ZD_LIB_PATH=$V/libzd_$2.so timeout -k 10 300 python bench.py --workload $3 --no-cpu-baseline --no-host-io > $out 2> ${out%.json}.err || exit 1
  fi
  python -c "import json; d=json.load(open('$out')); print('$1 $3', d['value'], d['ms_per_step'], {k: v for k, v in d['kernel_ms'].items() if v > 0.01}, d['verified_bit_exact'])"
}
for i in 1 2; do
  run new$i default c3s; run xreg4_$i xreg4 c3s; run xreg2_$i xreg2 c3s; run xreg1_$i xreg1 c3s
done
