#!/bin/bash
# r05 session 18: CSV fill addressed from the tile base (32-bit rooms, fewer
# SGPR spills, 6 waves / SIMD).
out=gpurun_out/r05_s18
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
step pytest_csv 400 $PYT tests/test_gpu_parser.py -k csv
step bench_csv 300 python -u bench.py --mode hbm --format csv --steps 10 --warmup 2
step bench_csv2 300 python -u bench.py --mode hbm --format csv --steps 10 --warmup 2
