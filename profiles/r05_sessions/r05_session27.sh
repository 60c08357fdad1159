#!/bin/bash
# r05 session 27: the hashed pass over resident text, one pass (look-back)
# against the counted path (DMLC_HASH_ONE_PASS=0).
out=gpurun_out/r05_s27
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
step hashed_onepass 400 python -u scripts/bench_hashed.py --sweep 256,1024 --steps 20
DMLC_HASH_ONE_PASS=0 step hashed_counted 400 python -u scripts/bench_hashed.py --sweep 256,1024 --steps 20
DMLC_HASH_ONE_PASS=0 step pytest_hashed_counted 400 python -u -m pytest -x -v --timeout 150 --timeout-method thread tests/test_gpu_hashed.py
