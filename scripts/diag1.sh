#!/bin/bash
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 60 tools/zd_diag tests/golden/resources/romeo.txt.zst gpurun_out/romeo.out > gpurun_out/diag_romeo.log 2>&1; echo "romeo rc=$?"
AMD_LOG_LEVEL=3 timeout -k 10 60 tools/zd_diag tests/golden/resources/welcome.zst > gpurun_out/diag_welcome.log 2>&1; echo "welcome rc=$?"
timeout -k 10 120 python -X faulthandler -c "
import torch; torch.zeros(1, device='cuda'); print('torch ok', flush=True)
import sys; sys.path[:0]=['.','zstd-decompressor_amd']
from zstd_decompressor.batch import Plan
p = Plan(open('tests/golden/resources/romeo.txt.zst','rb').read()); print('plan ok', p.info.nframes, flush=True)
" > gpurun_out/diag_py.log 2>&1; echo "py rc=$?"
tail -c 3000 gpurun_out/diag_welcome.log
