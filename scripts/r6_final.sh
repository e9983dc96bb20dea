#!/bin/bash
# Round-6 end check at HEAD: the whole GPU suite, smoke, the default bench
# line (C4), the c3s, C3, C2 and C5 level-1 lines, each step under its own limit.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp ZD_CORPUS_CACHE=/tmp/zdc
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/fin_pytest.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -2 gpurun_out/fin_pytest.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/fin_smoke.log 2>&1; rc=$?
echo "smoke rc=$rc"; tail -1 gpurun_out/fin_smoke.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python bench.py > gpurun_out/fin_c4.json 2> gpurun_out/fin_c4.err || exit 1
timeout -k 10 600 python bench.py --workload c3s > gpurun_out/fin_c3s.json 2> gpurun_out/fin_c3s.err || exit 1
timeout -k 10 600 python bench.py --workload c3 > gpurun_out/fin_c3.json 2> gpurun_out/fin_c3.err || exit 1
timeout -k 10 600 python bench.py --workload c2 > gpurun_out/fin_c2.json 2> gpurun_out/fin_c2.err || exit 1
timeout -k 10 600 python bench.py --workload c5 --level 1 > gpurun_out/fin_c5.json 2> gpurun_out/fin_c5.err || exit 1
for w in c4 c3s c3 c2 c5; do python -c "import json; d=json.load(open('gpurun_out/fin_$w.json')); print('$w', d['value'], d['ms_per_step'], d['roofline']['kernel'][:30], d['roofline']['kernel_ms'], d['roofline']['frac'], d['verified_bit_exact'], d['cpu_baseline']['value'])"; done
