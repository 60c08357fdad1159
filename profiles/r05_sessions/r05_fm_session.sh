#!/bin/bash
# r05 session on one box: fused HashedFM step, RecordIO chain count, CSV fill,
# transpose workspace.  A step whose tests fail does not stop the session; a
# time limit, abort or crash (GPU trouble) does.
out=gpurun_out/r05_fm
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
step pytest_rec 400 $PYT tests/test_gpu_recordio.py
step pytest_transpose 300 $PYT tests/test_gpu_ops.py -k transpose
step pytest_csv 400 $PYT tests -m gpu -k "csv or CSV"
step bench_csv 300 python -u bench.py --mode hbm --format csv --steps 10 --warmup 2
step bench_rec 300 python -u bench.py --mode hbm --format recordio --steps 10 --warmup 2
step bench_hashed 400 python -u scripts/bench_hashed.py --sweep "" --steps 20
step prof_hashed 400 bash -c "cd /tmp && rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$out/prof -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/scripts/bench_hashed.py --sweep '' --steps 10"
step prof_rec 400 bash -c "cd /tmp && rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$out/prof_rec -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --mode hbm --format recordio --steps 5 --warmup 2"
step bench_linear 400 python -u scripts/bench_linear.py
step csv_pricing 900 bash scripts/csv_pricing.sh r05_fm/csv
