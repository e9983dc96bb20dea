#!/bin/bash
# Round-end measurements on the GPU box, each step under its own time limit;
# stops at the first failure.  usage: scripts/round_profiles.sh TAG COMMIT
#   C4 bench line (CPU baseline included) + its rocprofv3 kernel stats +
#   FETCH_SIZE / WRITE_SIZE passes (profiles/traffic.json, stamped COMMIT);
#   C5 at levels 1 / 9 / 19, C2, C3 and the single-frame C3 with baselines.
#   PART=a: the C4 steps (+ SQ counters); PART=b: the other workloads (+ C3 kernel stats);
#   PART=c: one rank's share of C4 at 8 / 4 / 2 GPUs (each part fits one gpurun call).
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
step c4_prof 900 rocprofv3 --kernel-trace --stats -d gpurun_out/${tag}_prof_c4 -o run --output-format csv -- python bench.py --no-cpu-baseline --no-host-io &&
B="python bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-verify --no-host-io" &&
timeout -k 10 300 rocprofv3 --kernel-trace --pmc FETCH_SIZE -d gpurun_out/${tag}_pmc_fetch -o run --output-format csv -- $B > gpurun_out/${tag}_pmc_fetch.log 2>&1 &&
timeout -k 10 300 rocprofv3 --kernel-trace --pmc WRITE_SIZE -d gpurun_out/${tag}_pmc_write -o run --output-format csv -- $B > gpurun_out/${tag}_pmc_write.log 2>&1 &&
python scripts/pmc_traffic.py gpurun_out/${tag}_pmc_fetch gpurun_out/${tag}_pmc_write gpurun_out/${tag}_traffic.json "$commit" > /dev/null &&
timeout -k 10 300 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAVE_CYCLES SQ_WAIT_ANY -d gpurun_out/${tag}_pmc_sq -o run --output-format csv -- python bench.py --steps 1 --warmup 1 --unique-mib 512 --replicas 8 --no-cpu-baseline --no-verify --no-host-io > gpurun_out/${tag}_pmc_sq.log 2>&1 || exit 1
fi
if [[ $part == *b* ]]; then
step c5_L1 900 python bench.py --workload c5 --level 1 &&
step c5_L9 900 python bench.py --workload c5 --level 9 &&
step c5_L19 900 python bench.py --workload c5 --level 19 --unique-mib 256 --replicas 40 &&
step c2 600 python bench.py --workload c2 &&
step c3 600 python bench.py --workload c3 &&
step c3s 600 python bench.py --workload c3s &&
step c3_prof 600 rocprofv3 --kernel-trace --stats -d gpurun_out/${tag}_prof_c3 -o run --output-format csv -- python bench.py --workload c3 --no-cpu-baseline --no-host-io &&
step c3s_prof 600 rocprofv3 --kernel-trace --stats -d gpurun_out/${tag}_prof_c3s -o run --output-format csv -- python bench.py --workload c3s --no-cpu-baseline --no-host-io &&
step c2_1GiB 600 python bench.py --workload c2 --c2-mib 1024 --no-host-io &&
step frame_parse 300 python scripts/time_frame_parse.py || exit 1
fi
if [[ $part == *c* ]]; then       # one rank's share of the strong-scaled C4 on 8 / 4 / 2 GPUs, alone on one GPU
step share8 600 python bench.py --unique-mib 160 --replicas 8 --no-cpu-baseline --no-host-io &&
step share4 600 python bench.py --unique-mib 320 --replicas 8 --no-cpu-baseline --no-host-io &&
step share2 600 python bench.py --unique-mib 640 --replicas 8 --no-cpu-baseline --no-host-io || exit 1
fi
echo done
