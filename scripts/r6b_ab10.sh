#!/bin/bash
# Round-6 A/B 10: K4 with its block's symbols and code tables packed
# (ZD_K4_PACK: 1,636 B of LDS instead of 2,048; an OF table of AL 9 read from
# HBM), so more frames fit a CU: p17 (window 6,960 B: 9,216 B a wave, 17 a CU)
# and p18 (window 6,704 B, a 256-byte literal stage: 8,704 B, 18 a CU), against
# the default (9,856 B, 16 a CU).  Parity of p18 first.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp ZD_CORPUS_CACHE=/tmp/zdc
V=zstd-decompressor_amd/lib/variants
ZD_LIB_PATH=$V/libzd_p18.so timeout -k 10 700 python -u -m pytest -x -q --timeout 300 --timeout-method thread \
  tests/test_gpu_parity.py tests/test_fuzz.py -m gpu > gpurun_out/ab10_pytest.log 2>&1; rc=$?
echo "pytest p18 rc=$rc"; tail -2 gpurun_out/ab10_pytest.log
[ $rc -eq 0 ] || exit $rc
run() {   # run NAME LIB WORKLOAD [extra]
  local out=gpurun_out/ab10_$1_$3.json
  if [ "$2" = default ]; then
    timeout -k 10 300 python bench.py --workload $3 --no-cpu-baseline --no-host-io ${4:-} > $out 2> ${out%.json}.err || exit 1
  else
    ZD_LIB_PATH=$V/libzd_$2.so timeout -k 10 300 python bench.py --workload $3 --no-cpu-baseline --no-host-io ${4:-} > $out 2> ${out%.json}.err || exit 1
  fi
  python -c "import json; d=json.load(open('$out')); print('$1 $3', d['value'], d['ms_per_step'], {k: v for k, v in d['kernel_ms'].items() if v > 0.01}, d['roofline']['kernel_ms'], d['verified_bit_exact'])"
}
for i in 1 2; do
  run new$i default c4; run p17_$i p17 c4; run p18_$i p18 c4
done
run new1 default c5 "--level 1"; run p17_1 p17 c5 "--level 1"; run p18_1 p18 c5 "--level 1"
