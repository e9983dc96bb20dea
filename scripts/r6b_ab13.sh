#!/bin/bash
# Round-6 A/B 13: K3Q's window select by the qword first (ZD_K3Q_SEL2=1,
# lib/variants/libzd_sel2.so: 8 selects a step, not 10) against the default,
# on C4 and C5 L9; parity of the variant first.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp ZD_CORPUS_CACHE=/tmp/zdc
V=zstd-decompressor_amd/lib/variants
ZD_LIB_PATH=$V/libzd_sel2.so timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread \
  tests/test_gpu_parity.py "tests/test_fuzz.py::test_fuzz_structure_aware" -m gpu > gpurun_out/ab13_pytest.log 2>&1; rc=$?
echo "pytest sel2 rc=$rc"; tail -2 gpurun_out/ab13_pytest.log
[ $rc -eq 0 ] || exit $rc
run() {   # run NAME LIB WORKLOAD [extra]
  local out=gpurun_out/ab13_$1_$3.json
  if [ "$2" = default ]; then
    timeout -k 10 300 python bench.py --workload $3 --no-cpu-baseline --no-host-io ${4:-} > $out 2> ${out%.json}.err || exit 1
  else
    ZD_LIB_PATH=$V/libzd_$2.so timeout -k 10 300 python bench.py --workload $3 --no-cpu-baseline --no-host-io ${4:-} > $out 2> ${out%.json}.err || exit 1
  fi
  python -c "import json; d=json.load(open('$out')); print('$1 $3', d['value'], d['ms_per_step'], {k: v for k, v in d['kernel_ms'].items() if v > 0.01}, d['verified_bit_exact'])"
}
for i in 1 2; do
  run new$i default c4; run sel2_$i sel2 c4
done
run new1 default c5 "--level 9"; run sel2_1 sel2 c5 "--level 9"
