#!/bin/bash
# r05 session 22: RecordIO with 2 GiB replay pieces by default; tile-parser
# tests after the VGPR-base revert.
out=gpurun_out/r05_s22
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
step pytest_rec 400 $PYT tests/test_gpu_recordio.py tests/test_gpu_parser.py tests/test_gpu_hashed.py
step bench_rec 300 python -u bench.py --mode hbm --format recordio --steps 10 --warmup 2
step bench_rec2 300 python -u bench.py --mode hbm --format recordio --steps 10 --warmup 2
step bench_libsvm 300 python -u bench.py --mode hbm --steps 10 --warmup 2
