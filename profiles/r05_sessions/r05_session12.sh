#!/bin/bash
# r05 session 12: CSV positional tile counts (S1p) against the owning-tile
# count (DMLC_CSV_POSCOUNT=0).
out=gpurun_out/r05_s12
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
step bench_csv_pos 300 python -u bench.py --mode hbm --format csv --steps 10 --warmup 2
DMLC_CSV_POSCOUNT=0 step bench_csv_own 300 python -u bench.py --mode hbm --format csv --steps 10 --warmup 2
step prof_csv 400 bash -c "cd /tmp && rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$out/prof_csv -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --mode hbm --format csv --steps 5 --warmup 2"
