#!/bin/bash
# r05 checkpoint: headline bench, per-format HBM benches, hashed sweep, GPU suite.
out=gpurun_out/r05_final
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
step bench_default 400 python -u bench.py
step bench_libsvm_hbm 300 python -u bench.py --mode hbm --steps 10 --warmup 2
step bench_libfm_hbm 300 python -u bench.py --mode hbm --format libfm --steps 10 --warmup 2
step bench_csv_hbm 300 python -u bench.py --mode hbm --format csv --steps 10 --warmup 2
step bench_recordio_hbm 300 python -u bench.py --mode hbm --format recordio --steps 10 --warmup 2
step bench_hashed 600 python -u scripts/bench_hashed.py --sweep 128,256,512,1024,2048 --steps 20
step pytest_gpu 1000 python -u -m pytest -v --timeout 300 --timeout-method thread tests -m gpu
