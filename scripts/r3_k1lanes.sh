#!/bin/bash
# round 3: K1 lanes per workgroup on the fused C3 plan (K1's sequence half is on the critical path)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp ZD_CORPUS_CACHE=/tmp/zdc
for v in base sl8 sl24 base sl8 sl24; do
  if [ $v = base ]; then lib=zstd-decompressor_amd/lib/libzd.so; else lib=zstd-decompressor_amd/lib/variants/libzd_$v.so; fi
  ZD_LIB_PATH=$lib timeout -k 10 300 python bench.py --workload c3 --steps 5 --warmup 2 --no-cpu-baseline --no-host-io > gpurun_out/r3kl_$v.json 2>/dev/null; echo "c3 $v rc=$?"
  python -c "import json;d=json.load(open('gpurun_out/r3kl_$v.json'));print(d['value'],d['ms_per_step'],d['kernel_ms']['zd_k_tables'])"
done
