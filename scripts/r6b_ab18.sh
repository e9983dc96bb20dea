#!/bin/bash
# Round-6 A/B 18: the blocks' segment sums (zd_k_jsum_blocks) done inside zd_k_jprefix, one launch
# fewer (default build) against the two launches (lib/variants/libzd_jpunf.so, ZD_JP_FUSED=0) --
# K4J parity, c3s and C5 level-1 lines alternated, and the c3s kernel stats of the default build.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp ZD_CORPUS_CACHE=/tmp/zdc
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_large_frames.py \
  tests/test_fuzz.py "tests/test_gpu_parity.py::test_resources" "tests/test_gpu_parity.py::test_fused_table_builds" \
  "tests/test_gpu_parity.py::test_out_of_domain_triggers" "tests/test_gpu_parity.py::test_synthetic_multi_block_frames" "tests/test_gpu_parity.py::test_corrupted_inputs" "tests/test_gpu_parity.py::test_multi_block_frames_forked_plan" "tests/test_gpu_parity.py::test_context_block_by_block" "tests/test_gpu_parity.py::test_hip_graph_capture_replay" -m gpu > gpurun_out/ab18_pytest.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -2 gpurun_out/ab18_pytest.log
[ $rc -eq 0 ] || exit $rc
V=zstd-decompressor_amd/lib/variants
run() {   # run NAME LIB WORKLOAD [extra]
  local out=gpurun_out/ab18_$1_$3.json
  if [ "$2" = default ]; then
    timeout -k 10 300 python bench.py --workload $3 --no-cpu-baseline --no-host-io ${4:-} > $out 2> ${out%.json}.err || exit 1
  else
    ZD_LIB_PATH=$V/libzd_$2.so timeout -k 10 300 python bench.py --workload $3 --no-cpu-baseline --no-host-io ${4:-} > $out 2> ${out%.json}.err || exit 1
  fi
  python -c "import json; d=json.load(open('$out')); print('$1 $3', d['value'], d['ms_per_step'], d['roofline']['kernel_ms'], d['verified_bit_exact'])"
}
for i in 1 2 3; do run fused$i default c3s; run unf$i jpunf c3s; done
run fused1 default c5 "--level 1"; run unf1 jpunf c5 "--level 1"
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/ab18_prof_c3s -o run --output-format csv -- python bench.py --workload c3s --no-cpu-baseline --no-host-io > gpurun_out/ab18_prof.json 2> gpurun_out/ab18_prof.err || exit 1
python - <<'PY'
import csv, glob
f = glob.glob('gpurun_out/ab18_prof_c3s/**/*kernel_stats.csv', recursive=True)[0]
for r in csv.reader(open(f)):
    if r[0] != 'Name' and float(r[3]) > 10000:
        print(f"{r[0].split('(')[0][:45]:45s} {r[1]:>5s} {float(r[3])/1e3:9.1f} us")
PY
