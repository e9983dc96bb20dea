set -u
for v in fork nofork; do
  if [ $v = nofork ]; then export ZD_NO_FORK=1; fi
  ZD_CORPUS_CACHE=/tmp/zdc timeout -k 10 600 python bench.py --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/fork_$v.log 2>&1; rc=$?
  echo "== $v rc=$rc $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/fork_$v.log) $(grep -o '"verified_bit_exact": [a-z]*' gpurun_out/fork_$v.log)"
  [ $rc -eq 0 ] || exit $rc
done
