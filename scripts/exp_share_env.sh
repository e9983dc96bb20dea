#!/bin/bash
# One rank's share of C4 (bench.py --unique-mib M --replicas 8) with and without an
# environment setting, on one box.  usage: scripts/exp_share_env.sh M VAR=VALUE
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export ZD_CORPUS_CACHE=/tmp/zdc
m=$1; kv=$2
for e in "" "$kv"; do
  tag=${e:-default}; tag=${tag//[=,]/_}
  env $e timeout -k 10 600 python bench.py --unique-mib $m --replicas 8 --no-cpu-baseline --no-host-io \
    > gpurun_out/share_env_${m}_$tag.json 2> gpurun_out/share_env_${m}_$tag.err || exit 1
  echo "$m $tag done"
done
