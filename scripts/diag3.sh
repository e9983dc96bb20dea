#!/bin/bash
set -u
mkdir -p gpurun_out
timeout -k 10 120 python -X faulthandler -c "
import sys; sys.path[:0]=['.','zstd-decompressor_amd']
import numpy as np
from corpus import gen, libzstd
from oracle import oracle
print('imports ok', flush=True)
from zstd_decompressor.batch import decompress_status
for i in range(14):
    d = open(f'gpurun_in/kat{i}.zst','rb').read()
    print(i, oracle.decompress_status(d, False)[0], flush=True)
    print(i, decompress_status(d, False)[0], flush=True)
" > gpurun_out/diag_py3.log 2>&1; echo "py3 rc=$?"
tail -30 gpurun_out/diag_py3.log
AMD_LOG_LEVEL=3 timeout -k 10 300 python -m pytest tests/test_gpu_parity.py -x -q -s -p no:cacheprovider -k kat_frames > gpurun_out/diag_pytest.log 2>&1; echo "pytest rc=$?"
grep -v "^:3" gpurun_out/diag_pytest.log | tail -30
grep "^:" gpurun_out/diag_pytest.log | tail -15
