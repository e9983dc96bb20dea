set -u
cd "${GRAFT_REPO_ROOT:-.}"
export ZD_CORPUS_CACHE=/tmp/zdc
for cfg in "640" "320"; do
  for b in 1 0; do
    ZD_K3_BALANCE=$b timeout -k 10 600 python bench.py --unique-mib $cfg --replicas 8 --no-cpu-baseline --no-host-io > gpurun_out/bal_${cfg}_$b.json 2> gpurun_out/bal_${cfg}_$b.err || exit 1
    echo "cfg $cfg bal $b done"
  done
done
