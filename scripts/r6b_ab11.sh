#!/bin/bash
# Round-6 A/B 11: K4J with 12 hops a word in the sweeps after round 1 (the
# new default) -- parity of the K4J paths, then c3s against 16 / 24 sweep
# hops and against round 1 at 5 / 8 hops.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp ZD_CORPUS_CACHE=/tmp/zdc
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_large_frames.py \
  "tests/test_fuzz.py::test_fuzz_block_parallel" "tests/test_gpu_parity.py::test_resources" \
  "tests/test_gpu_parity.py::test_hip_graph_capture_replay" -m gpu > gpurun_out/ab11_pytest.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -2 gpurun_out/ab11_pytest.log
[ $rc -eq 0 ] || exit $rc
run() {   # run NAME WORKLOAD [extra]
  local out=gpurun_out/ab11_$1_$2.json
  timeout -k 10 300 python bench.py --workload $2 --no-cpu-baseline --no-host-io ${3:-} > $out 2> ${out%.json}.err || exit 1
  python -c "import json; d=json.load(open('$out')); print('$1 $2', d['value'], d['ms_per_step'], d['roofline']['kernel_ms'], d['verified_bit_exact'])"
}
for i in 1 2; do
  run new$i c3s
  ZD_J_HOPS2=16 run h16_$i c3s
  ZD_J_HOPS2=24 run h24_$i c3s
  ZD_J_HOPS=5 run r5_$i c3s
  ZD_J_HOPS=8 run r8_$i c3s
done
