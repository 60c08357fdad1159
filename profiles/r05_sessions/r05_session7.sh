#!/bin/bash
# r05 session 7: transpose with loads a batch / sub-tile ahead.
out=gpurun_out/r05_s7c
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
step pytest_transpose 400 $PYT tests/test_gpu_ops.py -k "transpose or gather or logreg or SpMV or spmv"
step bench_linear 400 python -u scripts/bench_linear.py
step prof_linear 400 bash -c "cd /tmp && rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$out/prof -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/scripts/bench_linear.py --iters 3"
