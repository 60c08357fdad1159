#!/bin/bash
# r05 session 10: decode-round slots of every other token (the five
# ds_read_b32 window reads of a 32-lane group spread over ~240 dwords).
out=gpurun_out/r05_s10
mkdir -p $out
export TMPDIR=/tmp
step() {  # name seconds cmd...
  local name=$1 secs=$2
  shift 2
  timeout -k 10 "$secs" "$@" > "$out/$name.log" 2>&1
  local rc=$?
  echo "$name rc=$rc"
  case $rc in 0|1) return 0 ;; *) echo "stopping after $name"; exit $rc ;; esac
}
PYT="python -u -m pytest -x -v --timeout 150 --timeout-method thread"
step pytest_tile 600 $PYT tests/test_gpu_parser.py tests/test_gpu_one_pass.py tests/test_gpu_hashed.py
step bench_libsvm 300 python -u bench.py --mode hbm --steps 10 --warmup 2
step bench_libfm 300 python -u bench.py --mode hbm --format libfm --steps 10 --warmup 2
step bench_hashed 300 python -u scripts/bench_hashed.py --sweep 256,1024 --steps 20
step pmc_libsvm 600 bash scripts/pmc_kernels.sh $out/pmc_libsvm python3 bench.py --mode hbm --steps 3 --warmup 1
