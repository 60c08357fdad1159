#!/bin/bash
# r05 session 21: larger merged replay pieces (fewer scan / finish / host
# turnarounds per epoch): RecordIO and LibSVM at --replay-chunk-mb 2048.
out=gpurun_out/r05_s21
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
step rec_1024 300 python -u bench.py --mode hbm --format recordio --steps 10 --warmup 2
step rec_2048 300 python -u bench.py --mode hbm --format recordio --steps 10 --warmup 2 --replay-chunk-mb 2048
step rec_2048b 300 python -u bench.py --mode hbm --format recordio --steps 10 --warmup 2 --replay-chunk-mb 2048
step libsvm_1536 300 python -u bench.py --mode hbm --steps 10 --warmup 2 --replay-chunk-mb 1536
step libsvm_2000 300 python -u bench.py --mode hbm --steps 10 --warmup 2 --replay-chunk-mb 2000
step csv_2000 300 python -u bench.py --mode hbm --format csv --steps 10 --warmup 2 --replay-chunk-mb 2000
