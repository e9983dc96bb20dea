#!/bin/bash
# PMC passes for the C4 kernels (one rocprofv3 run per counter group, each
# within the per-block slot limits of MI355X_MICROARCH.md), on C4 at
# UMIB MiB unique x REPS (default the full 1 GiB x 10).
# usage: scripts/pmc_all.sh TAG [UMIB REPS]
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
export ZD_CORPUS_CACHE=/tmp/zdc
tag=$1; umib=${2:-1024}; reps=${3:-10}
B="python bench.py --steps 1 --warmup 1 --unique-mib $umib --replicas $reps --no-cpu-baseline --no-verify"
timeout -k 10 120 rocprofv3 -L > gpurun_out/counters_list.txt 2>&1 || true
pass() {  # name counters...
  local name=$1; shift
  timeout -k 10 300 rocprofv3 --kernel-trace --pmc "$@" -d gpurun_out/pmc_${tag}_$name -o run --output-format csv -- $B > gpurun_out/pmc_${tag}_$name.log 2>&1
  local rc=$?
  echo "pmc $name rc=$rc"
  return $rc
}
pass sq SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAVE_CYCLES SQ_WAIT_ANY &&
pass sq2 SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SMEM SQ_INST_CYCLES_VMEM SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_BUSY_CYCLES &&
pass tcc TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum &&
pass fetch FETCH_SIZE &&
pass write WRITE_SIZE &&
pass grbm GRBM_GUI_ACTIVE GRBM_COUNT &&
python scripts/pmc_summary.py gpurun_out/pmc_${tag}_* > gpurun_out/pmc_${tag}_summary.txt
