# K4 batch phase cycles (ZD_K4_PROF builds): scripts/exp_k4prof.sh VARIANT... (default k4prof)
set -u
for v in "${@:-k4prof}"; do
ZD_LIB_PATH=zstd-decompressor_amd/lib/variants/libzd_$v.so timeout -k 10 300 python bench.py --steps 1 --warmup 1 --unique-mib 1024 --replicas 10 --no-cpu-baseline --no-verify --experiment --no-host-io --corpus-cache /tmp/zdc > gpurun_out/$v.log 2>&1; echo "$v rc=$?"
grep "^K4 frame" gpurun_out/$v.log | head -6
done
