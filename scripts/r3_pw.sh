#!/bin/bash
# the parallel-walk corruption inputs one by one through tools/decode_file
# (and its host-ASan build, tools/decode_file_asan, when present)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 120 python scripts/pw_inputs.py /tmp/pw || exit 1
for b in tools/decode_file tools/decode_file_asan; do
  [ -x $b ] || continue
  for f in /tmp/pw/pw_*.zst; do
    echo "== $b $f"
    ASAN_OPTIONS=detect_leaks=0:protect_shadow_gap=0 timeout -k 10 60 $b "$f" || { echo "rc=$?"; exit 1; }
  done
done
