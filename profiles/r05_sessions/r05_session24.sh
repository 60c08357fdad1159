#!/bin/bash
# r05 session 24: RecordIO stream mode with 4 KiB tiles (10 steps), then the
# end-of-round set (scripts/r05_final2.sh).
out=gpurun_out/r05_s24
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
step bench_rec_stream 300 python -u bench.py --format recordio --steps 10 --warmup 2
