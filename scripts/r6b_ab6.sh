#!/bin/bash
# Round-6 A/B 6: K4 with its blocks' symbols read from the FSE slots in HBM
# a batch ahead (ZD_K4_GSTAB=1), so a wave's LDS is 8 KiB and five waves fit
# per SIMD (lib/variants/libzd_gstab.so: 20 frames per CU, window 7,072 B),
# against the default (16 frames per CU, symbols in LDS); gstab4 is the same
# HBM symbol reads at four waves per SIMD with the 7,200-byte window.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp ZD_CORPUS_CACHE=/tmp/zdc
V=zstd-decompressor_amd/lib/variants
ZD_LIB_PATH=$V/libzd_gstab.so timeout -k 10 700 python -u -m pytest -x -q --timeout 300 --timeout-method thread \
  tests/test_gpu_parity.py tests/test_fuzz.py tests/test_frame_iterator.py -m gpu > gpurun_out/ab6_pytest.log 2>&1; rc=$?
echo "pytest gstab rc=$rc"; tail -2 gpurun_out/ab6_pytest.log
[ $rc -eq 0 ] || exit $rc
run() {   # run NAME LIB WORKLOAD [extra]
  local out=gpurun_out/ab6_$1_$3.json
  if [ "$2" = default ]; then
    timeout -k 10 300 python bench.py --workload $3 --no-cpu-baseline --no-host-io ${4:-} > $out 2> ${out%.json}.err || exit 1
  else
    ZD_LIB_PATH=$V/libzd_$2.so timeout -k 10 300 python bench.py --workload $3 --no-cpu-baseline --no-host-io ${4:-} > $out 2> ${out%.json}.err || exit 1
  fi
  python -c "import json; d=json.load(open('$out')); print('$1 $3', d['value'], d['ms_per_step'], {k: v for k, v in d['kernel_ms'].items() if v > 0.01}, d['roofline']['kernel_ms'], d['verified_bit_exact'])"
}
for i in 1 2; do
  run new$i default c4; run gstab_$i gstab c4; run gstab4_$i gstab4 c4
done
run new1 default c5 "--level 1"; run gstab_1 gstab c5 "--level 1"
run new1 default c3; run gstab_1 gstab c3
