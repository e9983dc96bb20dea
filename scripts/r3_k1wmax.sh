#!/bin/bash
# round 3: where the wave-per-block sequence tables pay (ZD_K1W_MAX: 0 = K1's lanes always)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp ZD_CORPUS_CACHE=/tmp/zdc
for m in 0 1000000 0 1000000; do
  ZD_K1W_MAX=$m timeout -k 10 300 python bench.py --unique-mib 160 --replicas 8 --steps 5 --warmup 2 --no-cpu-baseline --no-host-io > gpurun_out/r3kw_s8_$m.json 2>/dev/null; rc=$?
  echo "share8 k1w_max=$m rc=$rc $(python -c "import json;d=json.load(open('gpurun_out/r3kw_s8_$m.json'));print(d['value'],d['ms_per_step'],d.get('verified_bit_exact'),d.get('kernel_ms',{}).get('zd_k_tables'))")"; [ $rc = 0 ] || exit $rc
done
for m in 0 1000000; do
  ZD_K1W_MAX=$m timeout -k 10 400 python bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-host-io > gpurun_out/r3kw_c4_$m.json 2>/dev/null; rc=$?
  echo "c4 k1w_max=$m rc=$rc $(python -c "import json;d=json.load(open('gpurun_out/r3kw_c4_$m.json'));print(d['value'],d['ms_per_step'],d.get('verified_bit_exact'),d.get('kernel_ms',{}).get('zd_k_tables'))")"; [ $rc = 0 ] || exit $rc
done
