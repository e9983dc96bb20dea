#!/bin/bash
# Runs GPU steps on the gpurun box; each step has its own time limit and the
# script stops at the first fault/abort/timeout (exit 124/134/137/139 or
# negative signals).  Test failures (pytest exit 1) do not stop later steps.
# usage: scripts/gpu_run.sh STEP...   (steps: build test smoke bench prof pmc)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
export ZD_CORPUS_CACHE=${ZD_CORPUS_CACHE:-/tmp/zd_corpus}   # corpora shared by the steps of one call
fatal() { case "$1" in 124|134|137|139|132|135|136) return 0;; *) return 1;; esac; }
run() {  # name seconds cmd...
  local name=$1 secs=$2; shift 2
  echo "=== $name: $*" | tee -a gpurun_out/steps.log
  timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc" | tee -a gpurun_out/steps.log
  tail -5 "gpurun_out/$name.log"
  if fatal $rc; then echo "FATAL in $name, stopping"; exit $rc; fi
  return $rc
}
for s in "$@"; do
  case "$s" in
    build) run build 300 python -c "import __graft_entry__ as g; g.build()" || exit 1 ;;
    test)  run pytest 1100 python -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 300 --timeout-method thread ;;
    large) run pytest_large 900 python -u -m pytest -x -v -p no:cacheprovider --timeout 300 --timeout-method thread tests/test_large_frames.py tests/test_resource_digests.py "tests/test_gpu_parity.py::test_hip_graph_capture_replay" ;;
    testall) run pytest_all 1200 python -m pytest tests -m gpu -q -p no:cacheprovider ;;
    tail) run pytest_tail 1100 python -u -m pytest -x -v -p no:cacheprovider --timeout 900 --timeout-method thread -m gpu tests/test_k4f.py tests/test_large_frames.py tests/test_resource_digests.py tests/test_shard.py ;;
    t2) run pytest_t2 900 python -u -m pytest -x -v -p no:cacheprovider --timeout 600 --timeout-method thread "tests/test_gpu_parity.py::test_hip_graph_capture_replay" tests/test_shard.py tests/test_k4f.py -m gpu ;;
    benchc3s) run bench_c3s 600 python bench.py --workload c3s --steps 5 --warmup 2 --no-cpu-baseline ;;
    profc3s) run prof_c3s 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_c3s -o run --output-format csv -- python bench.py --workload c3s --steps 3 --warmup 1 --no-cpu-baseline ;;
    c3svar:*) v=${s#c3svar:}; ZD_LIB_PATH=zstd-decompressor_amd/lib/variants/libzd_$v.so run bench_c3s_$v 600 python bench.py --workload c3s --steps 5 --warmup 2 --no-cpu-baseline --no-host-io ;;
    profc3svar:*) v=${s#profc3svar:}; ZD_LIB_PATH=zstd-decompressor_amd/lib/variants/libzd_$v.so run prof_c3s_$v 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_c3s_$v -o run --output-format csv -- python bench.py --workload c3s --steps 3 --warmup 1 --no-cpu-baseline --no-host-io ;;
    pmcj) run pmc_j1 300 rocprofv3 --kernel-trace --kernel-include-regex "zd_k_jround|zd_k_jscatter" --pmc SQ_WAVES SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_SALU -d gpurun_out/pmc_j1 -o run --output-format csv -- python bench.py --workload c3s --steps 1 --warmup 1 --no-cpu-baseline --no-verify --no-host-io && run pmc_j2 300 rocprofv3 --kernel-trace --kernel-include-regex "zd_k_jround|zd_k_jscatter" --pmc TCC_HIT_sum TCC_MISS_sum TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum -d gpurun_out/pmc_j2 -o run --output-format csv -- python bench.py --workload c3s --steps 1 --warmup 1 --no-cpu-baseline --no-verify --no-host-io ;;
    c3senv:*) e=${s#c3senv:}; run bench_c3s_env_${e//[=,]/_} 600 env ${e//,/ } python bench.py --workload c3s --steps 5 --warmup 2 --no-cpu-baseline --no-host-io ;;
    fztrace) ZD_LIB_PATH=zstd-decompressor_amd/lib/variants/libzd_fztrace.so run fztrace 300 python scripts/fztrace.py ;;
    c3env:*) e=${s#c3env:}; run bench_c3_env_${e//[=,]/_} 600 env ${e//,/ } python bench.py --workload c3 --steps 10 --warmup 3 --no-cpu-baseline --no-host-io ;;
    c3var:*) v=${s#c3var:}; ZD_LIB_PATH=zstd-decompressor_amd/lib/variants/libzd_$v.so run bench_c3_$v 600 python bench.py --workload c3 --steps 10 --warmup 3 --no-cpu-baseline --no-host-io ;;
    c2bigvar:*) v=${s#c2bigvar:}; if [ "$v" = base ]; then lib=zstd-decompressor_amd/lib/libzd.so; else lib=zstd-decompressor_amd/lib/variants/libzd_$v.so; fi; ZD_LIB_PATH=$lib run bench_c2big_$v 600 python bench.py --workload c2 --c2-mib 1024 --steps 10 --warmup 3 --no-cpu-baseline --no-host-io ;;
    c2var:*) v=${s#c2var:}; if [ "$v" = base ]; then lib=zstd-decompressor_amd/lib/libzd.so; else lib=zstd-decompressor_amd/lib/variants/libzd_$v.so; fi; ZD_LIB_PATH=$lib run bench_c2_$v 600 python bench.py --workload c2 --steps 20 --warmup 5 --no-cpu-baseline --no-host-io ;;
    nofcs) run time_no_fcs 600 python -u scripts/time_no_fcs.py ;;
    nofcsvar:*) v=${s#nofcsvar:}; ZD_LIB_PATH=zstd-decompressor_amd/lib/variants/libzd_$v.so run time_no_fcs_$v 600 python -u scripts/time_no_fcs.py ;;
    benchc3) run bench_c3 600 python bench.py --workload c3 --steps 5 --warmup 2 --no-cpu-baseline ;;
    nofarq) ZD_LIB_PATH=zstd-decompressor_amd/lib/variants/libzd_nofar.so run bench_nofar 600 python bench.py --steps 3 --warmup 1 --unique-mib 256 --replicas 4 --no-cpu-baseline --no-verify --experiment --no-host-io ;;
    k3q8q) ZD_LIB_PATH=zstd-decompressor_amd/lib/variants/libzd_k3q8.so run bench_k3q8 600 python bench.py --steps 3 --warmup 1 --unique-mib 256 --replicas 4 --no-cpu-baseline --no-host-io ;;
    k3q8) ZD_LIB_PATH=zstd-decompressor_amd/lib/variants/libzd_k3q8.so run bench_k3q8_full 900 python bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-host-io ;;
    benchnc) run bench_nc 600 python bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-host-io ;;
    walk) run pytest_walk 600 python -u -m pytest -x -v -p no:cacheprovider --timeout 300 --timeout-method thread -m gpu tests/test_gpu_walk.py ;;
    smoke) run smoke 300 python -c "import __graft_entry__ as g; g.smoke()" ;;
    bench) run bench 900 python bench.py ;;
    benchq) run bench_quick 600 python bench.py --steps 3 --warmup 1 --unique-mib 256 --replicas 4 --no-cpu-baseline ;;
    prof) run prof 900 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python bench.py --steps 3 --warmup 1 --unique-mib 256 --replicas 4 --no-cpu-baseline ;;
    pmc) run pmc_sq 900 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAVE_CYCLES SQ_WAIT_ANY -d gpurun_out/pmc_sq -o run --output-format csv -- python bench.py --steps 1 --warmup 1 --unique-mib 256 --replicas 4 --no-cpu-baseline --no-verify ;;
    pmchbm) run pmc_fetch 900 rocprofv3 --kernel-trace --pmc FETCH_SIZE -d gpurun_out/pmc_fetch -o run --output-format csv -- python bench.py --steps 1 --warmup 1 --unique-mib 256 --replicas 4 --no-cpu-baseline --no-verify && run pmc_write 900 rocprofv3 --kernel-trace --pmc WRITE_SIZE -d gpurun_out/pmc_write -o run --output-format csv -- python bench.py --steps 1 --warmup 1 --unique-mib 256 --replicas 4 --no-cpu-baseline --no-verify ;;
    pmck2) run pmc_k2a 300 rocprofv3 --kernel-trace --kernel-include-regex "zd_k_huffman|zd_k_huf_pairs" --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAVE_CYCLES SQ_WAIT_ANY -d gpurun_out/pmc_k2a -o run --output-format csv -- python bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-verify --no-host-io && run pmc_k2b 300 rocprofv3 --kernel-trace --kernel-include-regex "zd_k_huffman" --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM -d gpurun_out/pmc_k2b -o run --output-format csv -- python bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-verify --no-host-io ;;
    varx:*) v=${s#varx:}; ZD_LIB_PATH=zstd-decompressor_amd/lib/variants/libzd_$v.so run bench_varx_$v 600 python bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-host-io --no-verify --experiment ;;
    prof10) run prof10 900 rocprofv3 --kernel-trace --stats -d gpurun_out/prof10 -o run --output-format csv -- python bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-host-io ;;
    pmc10) run pmc_sq10 600 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAVE_CYCLES SQ_WAIT_ANY -d gpurun_out/pmc_sq10 -o run --output-format csv -- python bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-verify --no-host-io ;;
    pmchbm10) run pmc_fetch10 600 rocprofv3 --kernel-trace --pmc FETCH_SIZE -d gpurun_out/pmc_fetch10 -o run --output-format csv -- python bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-verify --no-host-io && run pmc_write10 600 rocprofv3 --kernel-trace --pmc WRITE_SIZE -d gpurun_out/pmc_write10 -o run --output-format csv -- python bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-verify --no-host-io ;;
    benchc5:*) l=${s#benchc5:}; run bench_c5_L$l 900 python bench.py --workload c5 --level $l --no-host-io ;;
    benchc2) run bench_c2 600 python bench.py --workload c2 ;;
    benchc2big) run bench_c2_1GiB 600 python bench.py --workload c2 --c2-mib 1024 --no-cpu-baseline ;;
    profc2big) run prof_c2_1GiB 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_c2big -o run --output-format csv -- python bench.py --workload c2 --c2-mib 1024 --steps 3 --warmup 1 --no-cpu-baseline --no-host-io ;;
    share:*) x=${s#share:}; run bench_share_${x//\//of} 600 python bench.py --share $x --no-cpu-baseline --no-host-io ;;
    testvar:*) v=${s#testvar:}; ZD_LIB_PATH=zstd-decompressor_amd/lib/variants/libzd_$v.so run pytest_var_$v 1100 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread ;;
    k3g:*) v=${s#k3g:}; ZD_K3G=$v run bench_k3g_$v 600 python bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-host-io ;;
    c5var:*) v=${s#c5var:}; l=${v#*@}; v=${v%@*}; if [ "$v" = base ]; then lib=zstd-decompressor_amd/lib/libzd.so; else lib=zstd-decompressor_amd/lib/variants/libzd_$v.so; fi; ZD_LIB_PATH=$lib run bench_c5var_${v}_L$l 900 python bench.py --workload c5 --level $l --no-cpu-baseline --no-host-io ;;
    ovlp:*) n=${s#ovlp:}; run bench_ovlp_$n 600 python bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-host-io --overlap-streams $n ;;
    titer) run pytest_iter 300 python -u -m pytest -x -v -p no:cacheprovider --timeout 120 --timeout-method thread -m gpu tests/test_frame_iterator.py tests/test_lds_order.py ;;
    ldsorder) run lds_order 120 tools/lds_order_check 4096 256 ;;
    salub) run salu_bench 120 tools/salu_bench ;;
    testshard) run pytest_shard 600 python -u -m pytest -x -v -p no:cacheprovider --timeout 300 --timeout-method thread -m gpu tests/test_shard.py ;;
    env:*) e=${s#env:}; run bench_env_${e//[=,]/_} 600 env ${e//,/ } python bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-host-io ;;
    var:*) v=${s#var:}; ZD_LIB_PATH=zstd-decompressor_amd/lib/variants/libzd_$v.so run bench_var_$v 600 python bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-host-io ;;
    *) echo "unknown step $s"; exit 2 ;;
  esac
done
