#!/bin/bash
# r05 session 19: LibSVM / LibFM fill with its per-row output bases in VGPRs
# (SGPR spills 35 -> 29).
out=gpurun_out/r05_s19
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
step pytest_tile 600 $PYT tests/test_gpu_parser.py tests/test_gpu_one_pass.py tests/test_gpu_long_records.py
step bench_libsvm 300 python -u bench.py --mode hbm --steps 10 --warmup 2
step bench_libsvm2 300 python -u bench.py --mode hbm --steps 10 --warmup 2
step bench_libfm 300 python -u bench.py --mode hbm --format libfm --steps 10 --warmup 2
