#!/bin/bash
# Round-end measurements on the GPU box, each step under its own time limit;
# stops at the first failure.  usage: scripts/round_profiles.sh TAG COMMIT
#   C4 bench line (CPU baseline included) + its rocprofv3 kernel stats +
#   FETCH_SIZE / WRITE_SIZE passes (profiles/traffic.json, stamped COMMIT);
#   C5 at levels 1 / 9 / 19, C2, C3 and the single-frame C3 with baselines.
#   PART=a: the C4 steps only; PART=b: the other workloads only (each fits one gpurun call).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
export ZD_CORPUS_CACHE=/tmp/zdc
tag=$1; commit=$2
step() {  # name seconds cmd...
  local name=$1 secs=$2; shift 2
  timeout -k 10 "$secs" "$@" > "gpurun_out/${tag}_$name.json" 2> "gpurun_out/${tag}_$name.err"
  local rc=$?
  echo "$name rc=$rc"; tail -2 "gpurun_out/${tag}_$name.err"
  return $rc
}
part=${PART:-ab}
if [[ $part == *a* ]]; then
step c4 900 python bench.py &&
step c4_prof 900 rocprofv3 --kernel-trace --stats -d gpurun_out/${tag}_prof_c4 -o run --output-format csv -- python bench.py --no-cpu-baseline &&
B="python bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-verify" &&
timeout -k 10 300 rocprofv3 --kernel-trace --pmc FETCH_SIZE -d gpurun_out/${tag}_pmc_fetch -o run --output-format csv -- $B > gpurun_out/${tag}_pmc_fetch.log 2>&1 &&
timeout -k 10 300 rocprofv3 --kernel-trace --pmc WRITE_SIZE -d gpurun_out/${tag}_pmc_write -o run --output-format csv -- $B > gpurun_out/${tag}_pmc_write.log 2>&1 &&
python scripts/pmc_traffic.py gpurun_out/${tag}_pmc_fetch gpurun_out/${tag}_pmc_write gpurun_out/${tag}_traffic.json "$commit" > /dev/null || exit 1
fi
if [[ $part == *b* ]]; then
step c5_L1 900 python bench.py --workload c5 --level 1 &&
step c5_L9 900 python bench.py --workload c5 --level 9 &&
step c5_L19 900 python bench.py --workload c5 --level 19 --unique-mib 256 --replicas 40 &&
step c2 600 python bench.py --workload c2 &&
step c3 600 python bench.py --workload c3 &&
step c3s 600 python bench.py --workload c3s || exit 1
fi
echo done
