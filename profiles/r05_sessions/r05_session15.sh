#!/bin/bash
# r05 session 15: transpose bucket width (DMLC_T_LOWBITS 10 / 11 / 12 columns
# per bucket as a power of two): T4c cursor LDS vs T3 fan-out.
out=gpurun_out/r05_s15
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
for b in 10 11; do
  DMLC_T_LOWBITS=$b step pytest_ops_b$b 400 $PYT tests/test_gpu_ops.py -k "transpose or pairs or gather"
done
for b in 10 11 12; do
  DMLC_T_LOWBITS=$b step linear_b$b 300 python -u scripts/bench_linear.py --iters 5
done
for b in 10 12; do
  DMLC_T_LOWBITS=$b step prof_b$b 400 bash -c "cd /tmp && rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$out/prof_b$b -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/scripts/bench_linear.py --iters 3"
done
