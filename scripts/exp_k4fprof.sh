set -u
ZD_LIB_PATH=zstd-decompressor_amd/lib/variants/libzd_k4fprof.so timeout -k 10 300 python bench.py --steps 1 --warmup 1 --unique-mib 256 --replicas 1 --no-cpu-baseline --no-verify --experiment > gpurun_out/k4fprof.log 2>&1; echo rc=$?
grep "K4F" gpurun_out/k4fprof.log | head -40
