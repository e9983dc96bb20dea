#!/bin/bash
# Round-6 A/B 7: zd_decode_async's state reset as one kernel (default) against
# the six copy / fill launches (lib/variants/libzd_rcopies.so,
# ZD_RESET_COPIES); the whole GPU suite on the default build first.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp ZD_CORPUS_CACHE=/tmp/zdc
V=zstd-decompressor_amd/lib/variants
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/ab7_pytest.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -2 gpurun_out/ab7_pytest.log
[ $rc -eq 0 ] || exit $rc
run() {   # run NAME LIB WORKLOAD [extra]
  local out=gpurun_out/ab7_$1_$3.json
  if [ "$2" = default ]; then
    timeout -k 10 300 python bench.py --workload $3 --no-cpu-baseline --no-host-io ${4:-} > $out 2> ${out%.json}.err || exit 1
  else
    ZD_LIB_PATH=$V/libzd_$2.so timeout -k 10 300 python bench.py --workload $3 --no-cpu-baseline --no-host-io ${4:-} > $out 2> ${out%.json}.err || exit 1
  fi
  python -c "import json; d=json.load(open('$out')); print('$1 $3', d['value'], d['ms_per_step'], {k: v for k, v in d['kernel_ms'].items() if v > 0.01}, d['roofline']['kernel_ms'], d['verified_bit_exact'])"
}
for i in 1 2; do
  run new$i default c3s; run rc$i rcopies c3s
  run new$i default c3; run rc$i rcopies c3
  run new$i default c2; run rc$i rcopies c2
done
