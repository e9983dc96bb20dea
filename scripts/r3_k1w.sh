#!/bin/bash
# round 3: K1's sequence half one wave per block for plans of <= 8,192 tables; lighter K4J tail rounds
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp ZD_CORPUS_CACHE=/tmp/zdc
timeout -k 10 900 python -u -m pytest -x -v -p no:cacheprovider --timeout 300 --timeout-method thread tests -m gpu > gpurun_out/r3k1w_gpu.log 2>&1
rc=$?; echo "gpu suite rc=$rc"; grep -E "passed|failed|FAILED|Error" gpurun_out/r3k1w_gpu.log | tail -5; [ $rc = 0 ] || exit $rc
for w in c3s c3; do
  timeout -k 10 300 python bench.py --workload $w --steps 10 --warmup 3 --no-cpu-baseline --no-host-io > gpurun_out/r3k1w_$w.json 2>gpurun_out/r3k1w_$w.err; rc=$?
  echo "$w rc=$rc"; [ $rc = 0 ] || exit $rc
  python -c "import json;d=json.load(open('gpurun_out/r3k1w_$w.json'));print(d['value'],d['ms_per_step'],d.get('verified_bit_exact'),d.get('kernel_ms'))"
done
ZD_FUSE=0 timeout -k 10 300 python bench.py --workload c3 --steps 10 --warmup 3 --no-cpu-baseline --no-host-io > gpurun_out/r3k1w_c3nf.json 2>/dev/null; echo "c3 nofuse rc=$?"
python -c "import json;d=json.load(open('gpurun_out/r3k1w_c3nf.json'));print(d['value'],d['ms_per_step'],d.get('verified_bit_exact'))"
ZD_FUZZ_SEED=751 ZD_FUZZ_ITERS=4000 ZD_FUZZ_PLAN_ITERS=600 timeout -k 10 600 \
  python -u -m pytest tests/test_fuzz.py -v -s -p no:cacheprovider --timeout 550 --timeout-method thread > gpurun_out/fuzz_751.log 2>&1
rc=$?; echo "fuzz rc=$rc: $(grep -i 'outcome' gpurun_out/fuzz_751.log | tr '\n' ' ' | cut -c1-400) $(tail -1 gpurun_out/fuzz_751.log)"
