set -u
for g in ${GRIDS:-0 1024 1536 2048 3072}; do
  ZD_K4_GRID=$g ZD_LIB_PATH=${LIB:-zstd-decompressor_amd/lib/libzd.so} ZD_CORPUS_CACHE=/tmp/zdc timeout -k 10 600 python bench.py --steps 3 --warmup 1 --no-cpu-baseline --experiment > gpurun_out/grid_$g.log 2>&1; rc=$?
  echo "== grid $g rc=$rc $(grep -o '"kernel_ms": {[^}]*}' gpurun_out/grid_$g.log) $(grep -o '"verified_bit_exact": [a-z]*' gpurun_out/grid_$g.log)"
  [ $rc -eq 0 ] || exit $rc
done
