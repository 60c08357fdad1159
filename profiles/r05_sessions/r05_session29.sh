#!/bin/bash
# r05 session 29: counters (SQ / LDS / fetch / write) of the final RecordIO
# fill (4 KiB tiles) and the transpose kernels.
out=gpurun_out/r05_s29
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
step pmc_rec 700 bash scripts/pmc_kernels.sh $out/pmc_rec python3 bench.py --mode hbm --format recordio --steps 3 --warmup 1
step pmc_linear 700 bash scripts/pmc_kernels.sh $out/pmc_linear python3 scripts/bench_linear.py --iters 2
