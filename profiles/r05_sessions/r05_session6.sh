#!/bin/bash
# r05 session 6: counters of the transpose kernels and of the LibSVM fill.
out=gpurun_out/r05_s6
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
step pmc_linear 900 bash scripts/pmc_kernels.sh $out/pmc_linear python3 scripts/bench_linear.py --iters 2
step pmc_libsvm 600 bash scripts/pmc_kernels.sh $out/pmc_libsvm python3 bench.py --mode hbm --steps 3 --warmup 1 --no-prelaunch
