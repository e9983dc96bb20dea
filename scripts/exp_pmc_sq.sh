set -u
export TMPDIR=/tmp
B="python bench.py --steps 1 --warmup 1 --unique-mib 1024 --replicas 10 --no-cpu-baseline --no-verify --corpus-cache /tmp/zdc"
timeout -k 10 300 $B > gpurun_out/warm.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAVE_CYCLES SQ_WAIT_ANY -d gpurun_out/pmc_${1}_sq -o run --output-format csv -- $B > gpurun_out/pmc_${1}_sq.log 2>&1; echo "sq rc=$?"
timeout -k 10 300 rocprofv3 --kernel-trace --pmc SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INST_CYCLES_VMEM SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_BUSY_CYCLES SQ_INSTS_BRANCH -d gpurun_out/pmc_${1}_sq2 -o run --output-format csv -- $B > gpurun_out/pmc_${1}_sq2.log 2>&1; echo "sq2 rc=$?"
