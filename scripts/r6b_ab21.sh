#!/bin/bash
# Round-6 A/B 21: K4J round-1 hops per word (ZD_J_HOPS 4 / 5 / 6 default / 7 / 8) on c3s at HEAD,
# with the round-6 scan and sweep changes in; one build, the knob from the environment.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp ZD_CORPUS_CACHE=/tmp/zdc
for i in 1 2; do
  for h in 6 4 5 7 8; do
    out=gpurun_out/ab21_h${h}_$i.json
    ZD_J_HOPS=$h timeout -k 10 300 python bench.py --workload c3s --no-cpu-baseline --no-host-io > $out 2> ${out%.json}.err || exit 1
    python -c "import json; d=json.load(open('$out')); print('hops $h', d['value'], d['ms_per_step'], d['roofline']['kernel_ms'], d['verified_bit_exact'])"
  done
done
