#!/bin/bash
# r05 session 16: the 1024-column transpose default (ops / train tests, linear bench).
out=gpurun_out/r05_s16
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
step pytest_ops 400 $PYT tests/test_gpu_ops.py tests/test_gpu_train.py
step bench_linear 300 python -u scripts/bench_linear.py
