#!/bin/bash
# round 3: chain groups (K3 -> K4 per group) -- parity, then C3 / one-round plans with and without groups; K4 nt variant
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp ZD_CORPUS_CACHE=/tmp/zdc
timeout -k 10 600 python -u -m pytest -x -v -p no:cacheprovider --timeout 300 --timeout-method thread \
  tests/test_gpu_parity.py::test_chain_groups tests/test_gpu_parity.py::test_resources \
  tests/test_gpu_parity.py::test_corrupted_inputs_forked_plan "tests/test_gpu_parity.py::test_hip_graph_capture_replay" \
  tests/test_gpu_parity.py::test_one_round_plan tests/test_k4f.py > gpurun_out/r3g_t.log 2>&1
rc=$?; echo "tests rc=$rc"; grep -E "passed|failed|FAILED|Error" gpurun_out/r3g_t.log | tail -8
[ $rc -eq 0 ] || exit $rc
run() {  # name env... -- args
  local name=$1; shift
  env "$@" > gpurun_out/r3g_$name.json 2> gpurun_out/r3g_$name.err; local rc=$?
  echo "== $name rc=$rc"; python -c "import json,sys;d=json.load(open('gpurun_out/r3g_$name.json'));print(d['value'],d['ms_per_step'],d.get('kernel_ms'),d['verified_bit_exact'])" || tail -3 gpurun_out/r3g_$name.err
  return $rc
}
B="timeout -k 10 300 python bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-host-io"
for g in 1 3 2 1 3; do
  run c3_g$g ZD_GROUPS=$g $B --workload c3 || exit 1
  run share8_g$g ZD_GROUPS=$g $B --unique-mib 160 --replicas 8 || exit 1
done
bash scripts/bench_variants.sh base nt base nt
