#!/bin/bash
# r05 session 5: RecordIO next-epoch count beside the last fill, CSV single
# rounds + one-pass byte classes, full GPU suite.
out=gpurun_out/r05_s5
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
step bench_rec 300 python -u bench.py --mode hbm --format recordio --steps 10 --warmup 2
step prof_rec 400 bash -c "cd /tmp && rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$out/prof_rec -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --mode hbm --format recordio --steps 5 --warmup 2"
step bench_csv 300 python -u bench.py --mode hbm --format csv --steps 10 --warmup 2
step pmc_csv 600 bash scripts/pmc_kernels.sh $out/pmc_csv python3 bench.py --mode hbm --format csv --steps 3 --warmup 1 --no-prelaunch
step pytest_gpu 1000 python -u -m pytest -v --timeout 300 --timeout-method thread tests -m gpu
