#!/bin/bash
# round 3: K1's halves on two streams when K2 | K3 are not forked (ZD_K1FORK)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp ZD_CORPUS_CACHE=/tmp/zdc
timeout -k 10 900 python -u -m pytest -x -v -p no:cacheprovider --timeout 300 --timeout-method thread tests -m gpu > gpurun_out/r3k1f_gpu.log 2>&1
rc=$?; echo "gpu suite rc=$rc"; grep -E "passed|failed|FAILED|Error" gpurun_out/r3k1f_gpu.log | tail -5; [ $rc = 0 ] || exit $rc
for m in 0 1 0 1; do
  ZD_K1FORK=$m timeout -k 10 300 python bench.py --unique-mib 160 --replicas 8 --steps 5 --warmup 2 --no-cpu-baseline --no-host-io > gpurun_out/r3k1f_s8_$m.json 2>/dev/null; rc=$?
  echo "share8 k1fork=$m rc=$rc $(python -c "import json;d=json.load(open('gpurun_out/r3k1f_s8_$m.json'));print(d['value'],d['ms_per_step'],d.get('verified_bit_exact'))")"; [ $rc = 0 ] || exit $rc
done
for m in 0 1 0 1; do
  ZD_K1FORK=$m timeout -k 10 400 python bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-host-io > gpurun_out/r3k1f_c4_$m.json 2>/dev/null; rc=$?
  echo "c4 k1fork=$m rc=$rc $(python -c "import json;d=json.load(open('gpurun_out/r3k1f_c4_$m.json'));print(d['value'],d['ms_per_step'],d.get('verified_bit_exact'))")"; [ $rc = 0 ] || exit $rc
done
