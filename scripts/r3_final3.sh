#!/bin/bash
# round 3 final (zd_k_fused with its own sequence tables): GPU suite, smoke, fuzz, C3 bench + kernel stats, C4 bench
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp ZD_CORPUS_CACHE=/tmp/zdc
timeout -k 10 900 python -u -m pytest -x -v -p no:cacheprovider --timeout 300 --timeout-method thread \
  tests -m gpu > gpurun_out/r3_final3_gpu.log 2>&1
rc=$?; echo "gpu suite rc=$rc"; grep -E "passed|failed|FAILED|Error" gpurun_out/r3_final3_gpu.log | tail -5
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r3_final3_smoke.log 2>&1; rc=$?; echo "smoke rc=$rc"; tail -1 gpurun_out/r3_final3_smoke.log
[ $rc -eq 0 ] || exit $rc
for seed in 741 742; do
  ZD_FUZZ_SEED=$seed ZD_FUZZ_ITERS=6000 ZD_FUZZ_PLAN_ITERS=1000 timeout -k 10 600 \
    python -u -m pytest tests/test_fuzz.py -v -s -p no:cacheprovider --timeout 550 --timeout-method thread > gpurun_out/fuzz_$seed.log 2>&1
  rc=$?; echo "fuzz seed $seed rc=$rc: $(grep -i 'outcome' gpurun_out/fuzz_$seed.log | tr '\n' ' ' | cut -c1-300) $(tail -1 gpurun_out/fuzz_$seed.log)"
  [ $rc -eq 0 ] || exit $rc
done
timeout -k 10 600 python bench.py --workload c3 > gpurun_out/r3g_c3.json 2> gpurun_out/r3g_c3.err; echo "c3 rc=$?"
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/r3g_prof_c3 -o run --output-format csv -- python bench.py --workload c3 --no-cpu-baseline --no-host-io > gpurun_out/r3g_c3_prof.log 2>&1; echo "c3 prof rc=$?"
timeout -k 10 900 python bench.py > gpurun_out/r3g_c4.json 2> gpurun_out/r3g_c4.err; echo "c4 rc=$?"
