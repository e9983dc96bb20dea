#!/bin/bash
# Round-6 A/B 8: K3L building its blocks' sequence tables (zd_k_sequences_ls, default) against
# K1's sequence half launched ahead of K3L (lib/variants/libzd_sel0.so, ZD_K3L_SELF=0);
# the whole GPU suite on the default build first.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp ZD_CORPUS_CACHE=/tmp/zdc
V=zstd-decompressor_amd/lib/variants
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/ab8_pytest.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -2 gpurun_out/ab8_pytest.log
[ $rc -eq 0 ] || exit $rc
run() {   # run NAME LIB WORKLOAD [extra]
  local out=gpurun_out/ab8_$1_$3.json
  if [ "$2" = default ]; then
    timeout -k 10 300 python bench.py --workload $3 --no-cpu-baseline --no-host-io ${4:-} > $out 2> ${out%.json}.err || exit 1
  else
    ZD_LIB_PATH=$V/libzd_$2.so timeout -k 10 300 python bench.py --workload $3 --no-cpu-baseline --no-host-io ${4:-} > $out 2> ${out%.json}.err || exit 1
  fi
  python -c "import json; d=json.load(open('$out')); print('$1 $3', d['value'], d['ms_per_step'], {k: v for k, v in d['kernel_ms'].items() if v > 0.01}, d['roofline']['kernel_ms'], d['verified_bit_exact'])"
}
for i in 1 2 3; do
  run new$i default c3s; run sel0_$i sel0 c3s
  run new$i default c3; run sel0_$i sel0 c3
done
