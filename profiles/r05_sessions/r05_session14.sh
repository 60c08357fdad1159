#!/bin/bash
# r05 session 14: T4c write frontier -- the transpose build with T4c
# throttled by extra LDS per wave (DMLC_T4C_LDS bytes: 10 / 5 / 3 / 2 / 1
# waves per CU).
out=gpurun_out/r05_s14
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
for l in 0 16384 36864 65536 131072; do
  DMLC_T4C_LDS=$l step linear_lds$l 300 python -u scripts/bench_linear.py --iters 5
done
