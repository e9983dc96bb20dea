#!/bin/bash
# round 3: K1 sequence half three lanes per block (parity + C3 / one-round plans), kernel trace of grouped C3
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp ZD_CORPUS_CACHE=/tmp/zdc
timeout -k 10 600 python -u -m pytest -x -v -p no:cacheprovider --timeout 300 --timeout-method thread \
  tests/test_gpu_parity.py::test_chain_groups tests/test_gpu_parity.py::test_resources \
  tests/test_gpu_parity.py::test_corrupted_inputs_forked_plan tests/test_gpu_parity.py::test_multi_block_frames_forked_plan \
  tests/test_gpu_parity.py::test_one_round_plan tests/test_gpu_parity.py::test_k1_large_tables tests/test_fuzz.py > gpurun_out/r3t_t.log 2>&1
rc=$?; echo "tests rc=$rc"; grep -E "passed|failed|FAILED|Error" gpurun_out/r3t_t.log | tail -8
[ $rc -eq 0 ] || exit $rc
B="timeout -k 10 300 python bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-host-io"
for g in 1 3; do
  ZD_GROUPS=$g $B --workload c3 > gpurun_out/r3t_c3_g$g.json 2>/dev/null; echo "c3 g$g rc=$?"; cat gpurun_out/r3t_c3_g$g.json | head -c 300; echo
  ZD_GROUPS=$g $B --unique-mib 160 --replicas 8 > gpurun_out/r3t_s8_g$g.json 2>/dev/null; echo "s8 g$g rc=$?"; cat gpurun_out/r3t_s8_g$g.json | head -c 300; echo
done
ZD_GROUPS=3 timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/r3t_trace -o run --output-format csv -- python bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-host-io --workload c3 > gpurun_out/r3t_trace.log 2>&1; echo "trace rc=$?"
