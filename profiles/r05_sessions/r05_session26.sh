#!/bin/bash
# r05 session 26: T3 row search by an LDS histogram + DPP scan (was a chain
# of six bpermutes per group).
out=gpurun_out/r05_s26
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
step bench_linear2 300 python -u scripts/bench_linear.py
step prof_linear 400 bash -c "cd /tmp && rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$out/prof_linear -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/scripts/bench_linear.py --iters 3"
