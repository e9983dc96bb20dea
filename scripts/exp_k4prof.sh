set -u
ZD_LIB_PATH=zstd-decompressor_amd/lib/variants/libzd_k4prof.so timeout -k 10 300 python bench.py --steps 1 --warmup 1 --unique-mib 1024 --replicas 10 --no-cpu-baseline --no-verify --experiment --corpus-cache /tmp/zdc > gpurun_out/k4prof.log 2>&1; echo rc=$?
grep "^K4 frame" gpurun_out/k4prof.log | head -12
