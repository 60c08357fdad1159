#!/bin/bash
# r05 session 23: RecordIO 4 KiB tiles (fill: 68 VGPRs, 20 KiB LDS, 7 waves /
# SIMD instead of 4).
out=gpurun_out/r05_s23
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
step pytest_rec 400 $PYT tests/test_gpu_recordio.py
step bench_rec 300 python -u bench.py --mode hbm --format recordio --steps 10 --warmup 2
step bench_rec2 300 python -u bench.py --mode hbm --format recordio --steps 10 --warmup 2
step bench_rec_stream 300 python -u bench.py --format recordio --steps 3 --warmup 1
step prof_rec 400 bash -c "cd /tmp && rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$out/prof_rec -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --mode hbm --format recordio --steps 5 --warmup 2"
