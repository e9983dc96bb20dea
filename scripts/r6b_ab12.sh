#!/bin/bash
# Round-6 A/B 12: K4J's value decode (zd_k_jsum, zd_k_jscatter) with the LL / ML code tables in LDS
# (default) against ll_code / ml_code arithmetic (lib/variants/libzd_jcl0.so,
# ZD_J_CODELUT=0); K4J parity first.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp ZD_CORPUS_CACHE=/tmp/zdc
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_large_frames.py \
  "tests/test_fuzz.py::test_fuzz_block_parallel" "tests/test_gpu_parity.py::test_resources" \
  "tests/test_gpu_parity.py::test_hip_graph_capture_replay" -m gpu > gpurun_out/ab12_pytest.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -2 gpurun_out/ab12_pytest.log
[ $rc -eq 0 ] || exit $rc
run() {   # run NAME WORKLOAD [extra]
  local out=gpurun_out/ab12_$1_$2.json
  timeout -k 10 300 python bench.py --workload $2 --no-cpu-baseline --no-host-io ${3:-} > $out 2> ${out%.json}.err || exit 1
  python -c "import json; d=json.load(open('$out')); print('$1 $2', d['value'], d['ms_per_step'], d['roofline']['kernel_ms'], d['verified_bit_exact'])"
}
V=zstd-decompressor_amd/lib/variants
for i in 1 2 3; do
  run new$i c3s
  ZD_LIB_PATH=$V/libzd_jcl0.so run jcl0_$i c3s
done
