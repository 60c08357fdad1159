#!/bin/bash
# r05 session 20: hash kernel with its per-row output bases in VGPRs.
out=gpurun_out/r05_s20
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
step pytest_hashed 400 $PYT tests/test_gpu_hashed.py
step bench_hashed 400 python -u scripts/bench_hashed.py --sweep 256,1024 --steps 20
step bench_hashed2 400 python -u scripts/bench_hashed.py --sweep 256,1024 --steps 20
