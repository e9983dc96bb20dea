set -u
bash scripts/gpu_run.sh test || exit 1
UMIB=1024 REPS=10 bash scripts/bench_variants.sh base k3nt k3w2 k3w2nt || exit 1
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --pmc TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_TRANSLATION_HIT_sum -d gpurun_out/pmc_tcp -o run --output-format csv -- python bench.py --steps 1 --warmup 1 --unique-mib 1024 --replicas 10 --no-cpu-baseline --no-verify --corpus-cache /tmp/zdc > gpurun_out/pmc_tcp.log 2>&1; echo "tcp rc=$?"
