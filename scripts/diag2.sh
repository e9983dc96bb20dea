#!/bin/bash
set -u
mkdir -p gpurun_out
for i in 0 1 2 3 4 5 6 7 8 9 10 11 12 13; do
  timeout -k 10 60 tools/zd_diag gpurun_in/kat$i.zst > gpurun_out/diag_kat$i.log 2>&1; rc=$?; echo "kat$i rc=$rc"
  case $rc in 124|134|137|139) echo stop; break;; esac
done
timeout -k 10 120 python -X faulthandler -c "
import sys; sys.path[:0]=['.','zstd-decompressor_amd']
from zstd_decompressor.batch import Plan
p = Plan(open('tests/golden/resources/romeo.txt.zst','rb').read()); print('plan ok', p.info.nframes, flush=True)
p = Plan(open('gpurun_in/kat0.zst','rb').read()); print('plan ok', p.info.nframes, flush=True)
" > gpurun_out/diag_py2.log 2>&1; echo "py rc=$?"
cat gpurun_out/diag_py2.log | head -20
