#!/bin/bash
# round 3: K4 phase profile (ZD_K4_PROF variant), SQ counters on C4 4 GiB, FETCH_SIZE calibration
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp ZD_CORPUS_CACHE=/tmp/zdc
B="python bench.py --steps 1 --warmup 1 --unique-mib 256 --replicas 4 --no-cpu-baseline --no-host-io"
ZD_LIB_PATH=zstd-decompressor_amd/lib/variants/libzd_k4prof.so timeout -k 10 300 $B --experiment > gpurun_out/r3e_k4prof.log 2>&1; echo "k4prof rc=$?"
grep "K4 frame" gpurun_out/r3e_k4prof.log | head -6
timeout -k 10 300 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAVE_CYCLES SQ_WAIT_ANY -d gpurun_out/r3e_pmc_sq -o run --output-format csv -- $B --no-verify > gpurun_out/r3e_pmc_sq.log 2>&1; echo "pmc sq rc=$?"
timeout -k 10 120 rocprofv3 --kernel-trace --pmc FETCH_SIZE -d gpurun_out/r3e_calib_fetch -o run --output-format csv -- tools/fetch_calib > gpurun_out/r3e_calib.log 2>&1; echo "calib rc=$?"
timeout -k 10 120 rocprofv3 --kernel-trace --pmc TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum -d gpurun_out/r3e_calib_req -o run --output-format csv -- tools/fetch_calib > gpurun_out/r3e_calib2.log 2>&1; echo "calib2 rc=$?"
bash scripts/bench_variants.sh base rl stsb base rl stsb
