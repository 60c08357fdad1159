#!/bin/bash
# r05 session 3: fused FM step with one barrier per tile.
out=gpurun_out/r05_s3
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
step pytest_fm 400 $PYT tests/test_gpu_hashed.py -k "fm_"
step bench_hashed 400 python -u scripts/bench_hashed.py --sweep "" --steps 20
step prof_hashed 400 bash -c "cd /tmp && rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$out/prof -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/scripts/bench_hashed.py --sweep '' --steps 10"
step pmc_fm 600 bash scripts/pmc_kernels.sh $out/pmc_fm python3 scripts/bench_hashed.py --sweep "" --steps 3
