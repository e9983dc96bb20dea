#!/bin/bash
# Round-6 A/B 20: K4J segment sums two segments a wave (default, ZD_JSUM_P=2: a run of one block's
# segments shares the block's tables and one record stream) against one (libzd_jsp1.so, the old
# launch) and four (libzd_jsp4.so) -- K4J parity of the default and P=4, c3s and C5 level-1 lines
# alternated, c3s kernel stats of the default.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp ZD_CORPUS_CACHE=/tmp/zdc
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_large_frames.py \
  tests/test_fuzz.py "tests/test_gpu_parity.py::test_resources" "tests/test_gpu_parity.py::test_fused_table_builds" \
  "tests/test_gpu_parity.py::test_out_of_domain_triggers" "tests/test_gpu_parity.py::test_synthetic_multi_block_frames" "tests/test_gpu_parity.py::test_corrupted_inputs" "tests/test_gpu_parity.py::test_multi_block_frames_forked_plan" "tests/test_gpu_parity.py::test_context_block_by_block" "tests/test_gpu_parity.py::test_hip_graph_capture_replay" -m gpu > gpurun_out/ab20_pytestdef.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -2 gpurun_out/ab20_pytestdef.log
[ $rc -eq 0 ] || exit $rc
ZD_LIB_PATH=zstd-decompressor_amd/lib/variants/libzd_jsp4.so timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_large_frames.py \
  tests/test_fuzz.py "tests/test_gpu_parity.py::test_resources" "tests/test_gpu_parity.py::test_fused_table_builds" \
  "tests/test_gpu_parity.py::test_out_of_domain_triggers" "tests/test_gpu_parity.py::test_synthetic_multi_block_frames" "tests/test_gpu_parity.py::test_corrupted_inputs" "tests/test_gpu_parity.py::test_multi_block_frames_forked_plan" "tests/test_gpu_parity.py::test_context_block_by_block" "tests/test_gpu_parity.py::test_hip_graph_capture_replay" -m gpu > gpurun_out/ab20_pytest4.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -2 gpurun_out/ab20_pytest4.log
[ $rc -eq 0 ] || exit $rc
V=zstd-decompressor_amd/lib/variants
run() {   # run NAME LIB WORKLOAD [extra]
  local out=gpurun_out/ab20_$1_$3.json
  if [ "$2" = default ]; then
    timeout -k 10 300 python bench.py --workload $3 --no-cpu-baseline --no-host-io ${4:-} > $out 2> ${out%.json}.err || exit 1
  else
    ZD_LIB_PATH=$V/libzd_$2.so timeout -k 10 300 python bench.py --workload $3 --no-cpu-baseline --no-host-io ${4:-} > $out 2> ${out%.json}.err || exit 1
  fi
  python -c "import json; d=json.load(open('$out')); print('$1 $3', d['value'], d['ms_per_step'], d['roofline']['kernel_ms'], d['verified_bit_exact'])"
}
for i in 1 2 3; do run p2_$i default c3s; run p1_$i jsp1 c3s; run p4_$i jsp4 c3s; done
run p2_1 default c5 "--level 1"; run p1_1 jsp1 c5 "--level 1"; run p4_1 jsp4 c5 "--level 1"

timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/ab20_prof_c3s -o run --output-format csv -- python bench.py --workload c3s --no-cpu-baseline --no-host-io > gpurun_out/ab20_prof.json 2> gpurun_out/ab20_prof.err || exit 1
python - <<'PY'
import csv, glob
f = glob.glob('gpurun_out/ab20_prof_c3s/**/*kernel_stats.csv', recursive=True)[0]
for r in csv.reader(open(f)):
    if r[0] != 'Name' and 'zd_k_j' in r[0]:
        print(f"{r[0].split('(')[0][:45]:45s} {r[1]:>5s} {float(r[3])/1e3:9.1f} us")
PY
