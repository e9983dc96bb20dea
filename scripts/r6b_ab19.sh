#!/bin/bash
# Round-6 A/B 19: K4J scatter segments of 384 and 768 sequences (lib/variants/libzd_jseg384.so,
# libzd_jseg768.so, ZD_J_SEG) against 512 (default) -- K4J parity of both variants, c3s and C5
# level-1 lines alternated.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp ZD_CORPUS_CACHE=/tmp/zdc
ZD_LIB_PATH=zstd-decompressor_amd/lib/variants/libzd_jseg384.so timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_large_frames.py \
  tests/test_fuzz.py "tests/test_gpu_parity.py::test_resources" "tests/test_gpu_parity.py::test_fused_table_builds" \
  "tests/test_gpu_parity.py::test_out_of_domain_triggers" "tests/test_gpu_parity.py::test_synthetic_multi_block_frames" "tests/test_gpu_parity.py::test_corrupted_inputs" "tests/test_gpu_parity.py::test_multi_block_frames_forked_plan" "tests/test_gpu_parity.py::test_context_block_by_block" "tests/test_gpu_parity.py::test_hip_graph_capture_replay" -m gpu > gpurun_out/ab19_pytest384.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -2 gpurun_out/ab19_pytest384.log
[ $rc -eq 0 ] || exit $rc
ZD_LIB_PATH=zstd-decompressor_amd/lib/variants/libzd_jseg768.so timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_large_frames.py \
  tests/test_fuzz.py "tests/test_gpu_parity.py::test_resources" "tests/test_gpu_parity.py::test_fused_table_builds" \
  "tests/test_gpu_parity.py::test_out_of_domain_triggers" "tests/test_gpu_parity.py::test_synthetic_multi_block_frames" "tests/test_gpu_parity.py::test_corrupted_inputs" "tests/test_gpu_parity.py::test_multi_block_frames_forked_plan" "tests/test_gpu_parity.py::test_context_block_by_block" "tests/test_gpu_parity.py::test_hip_graph_capture_replay" -m gpu > gpurun_out/ab19_pytest768.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -2 gpurun_out/ab19_pytest768.log
[ $rc -eq 0 ] || exit $rc
V=zstd-decompressor_amd/lib/variants
run() {   # run NAME LIB WORKLOAD [extra]
  local out=gpurun_out/ab19_$1_$3.json
  if [ "$2" = default ]; then
    timeout -k 10 300 python bench.py --workload $3 --no-cpu-baseline --no-host-io ${4:-} > $out 2> ${out%.json}.err || exit 1
  else
    ZD_LIB_PATH=$V/libzd_$2.so timeout -k 10 300 python bench.py --workload $3 --no-cpu-baseline --no-host-io ${4:-} > $out 2> ${out%.json}.err || exit 1
  fi
  python -c "import json; d=json.load(open('$out')); print('$1 $3', d['value'], d['ms_per_step'], d['roofline']['kernel_ms'], d['verified_bit_exact'])"
}
for i in 1 2 3; do run s512_$i default c3s; run s384_$i jseg384 c3s; run s768_$i jseg768 c3s; done
run s512_1 default c5 "--level 1"; run s384_1 jseg384 c5 "--level 1"; run s768_1 jseg768 c5 "--level 1"
