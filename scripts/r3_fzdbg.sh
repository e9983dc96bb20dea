#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
echo "== K4F off, no fuse (streaming K4 on C3 frames)"; CASES=plain ZD_K4F=0 timeout -k 10 300 python scripts/fz_debug.py 2>&1 | grep -v amdgpu.ids
echo "== K4F default"; CASES=plain timeout -k 10 300 python scripts/fz_debug.py 2>&1 | grep -v amdgpu.ids
echo "== fused"; CASES=all timeout -k 10 300 python scripts/fz_debug.py 2>&1 | grep -v amdgpu.ids
