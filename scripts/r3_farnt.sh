#!/bin/bash
# round 3: parity after reverting chain groups / seq3; nontemporal far-match loads past a distance
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp ZD_CORPUS_CACHE=/tmp/zdc
timeout -k 10 600 python -u -m pytest -x -v -p no:cacheprovider --timeout 300 --timeout-method thread \
  tests/test_gpu_parity.py::test_mixed_frame_plans tests/test_gpu_parity.py::test_resources \
  tests/test_gpu_parity.py::test_corrupted_inputs_forked_plan "tests/test_gpu_parity.py::test_hip_graph_capture_replay" > gpurun_out/r3f_t.log 2>&1
rc=$?; echo "tests rc=$rc"; grep -E "passed|failed|FAILED|Error" gpurun_out/r3f_t.log | tail -8
[ $rc -eq 0 ] || exit $rc
bash scripts/bench_variants.sh base farnt4096 farnt16384 farnt65536 base farnt4096 farnt16384 farnt65536
