#!/bin/bash
# r05 session 28: bucket width 2^10 vs 2^11 after the T3 / T4c changes.
out=gpurun_out/r05_s28
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
for b in 10 11 10 11; do
  DMLC_T_LOWBITS=$b step linear_b${b}_$RANDOM 300 python -u scripts/bench_linear.py --iters 10
done
