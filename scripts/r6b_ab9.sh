#!/bin/bash
# Round-6 A/B 9: the timed steps replayed from a captured HIP graph (bench.py
# --graph) against launched per step (the default), on c3s, C3, C2 and C4;
# then the Frame.parse step timing.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp ZD_CORPUS_CACHE=/tmp/zdc
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread \
  "tests/test_gpu_parity.py::test_hip_graph_capture_replay" -m gpu > gpurun_out/ab9_pytest.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -2 gpurun_out/ab9_pytest.log
[ $rc -eq 0 ] || exit $rc
run() {   # run NAME WORKLOAD [extra]
  local out=gpurun_out/ab9_$1_$2.json
  timeout -k 10 300 python bench.py --workload $2 --no-cpu-baseline --no-host-io ${3:-} > $out 2> ${out%.json}.err || exit 1
  python -c "import json; d=json.load(open('$out')); print('$1 $2', d['value'], d['ms_per_step'], d['roofline']['kernel_ms'], d['verified_bit_exact'], d['config'].get('step'))"
}
for i in 1 2; do
  run graph$i c3s --graph; run launch$i c3s
  run graph$i c3 --graph; run launch$i c3
  run graph$i c2 --graph; run launch$i c2
done
run graph1 c4 --graph; run launch1 c4
timeout -k 10 300 python scripts/time_frame_parse.py gpurun_out/ab9_frame_parse.json || exit 1
# the default bench lines (launched per step, CPU baselines included)
for w in c3 c3s c2; do
  timeout -k 10 600 python bench.py --workload $w > gpurun_out/ab9_full_$w.json 2> gpurun_out/ab9_full_$w.err || exit 1
done
# hops in the sweeps after round 1 (ZD_J_HOPS2; round 1 keeps 6)
for h in 4 8 12; do
  ZD_J_HOPS2=$h run hops2_$h c3s
done
