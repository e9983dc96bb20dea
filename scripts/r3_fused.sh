#!/bin/bash
# round 3: zd_k_fused (K3 + K4 per group of four frames) -- parity, then C3 fused vs two launches, C4 unchanged
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp ZD_CORPUS_CACHE=/tmp/zdc
timeout -k 10 600 python -u -m pytest -x -v -p no:cacheprovider --timeout 300 --timeout-method thread \
  tests/test_gpu_parity.py::test_fused_plans tests/test_gpu_parity.py::test_resources \
  tests/test_gpu_parity.py::test_corrupted_inputs_forked_plan tests/test_gpu_parity.py::test_mixed_frame_plans \
  "tests/test_gpu_parity.py::test_hip_graph_capture_replay" > gpurun_out/r3fz_t.log 2>&1
rc=$?; echo "tests rc=$rc"; grep -E "passed|failed|FAILED|Error|assert" gpurun_out/r3fz_t.log | tail -8
[ $rc -eq 0 ] || exit $rc
B="timeout -k 10 300 python bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-host-io"
for fz in 0 1 1; do
  ZD_FUSE=$fz $B --workload c3 > gpurun_out/r3fz_c3_$fz.json 2>/dev/null; echo "c3 fuse=$fz rc=$?"
  python -c "import json;d=json.load(open('gpurun_out/r3fz_c3_$fz.json'));print(d['value'],d['ms_per_step'],d['verified_bit_exact'])"
done
bash scripts/bench_variants.sh base
ZD_FUSE=1 timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/r3fz_trace -o run --output-format csv -- python bench.py --workload c3 --steps 2 --warmup 1 --no-cpu-baseline --no-host-io > gpurun_out/r3fz_trace.log 2>&1; echo "trace rc=$?"
