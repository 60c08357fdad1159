#!/usr/bin/env bash
# End-of-round GPU session: the whole GPU suite, smoke(), the headline bench
# (default N=1 run) under rocprofv3 --stats, the HBM / hashed / FM benches
# and the https remote reader.  Every GPU step has its own time limit; the
# first failure ends the script.   OUT=gpurun_out/final bash scripts/final_session.sh
set -u
OUT=${OUT:-gpurun_out/final}
mkdir -p "$OUT"
export TMPDIR=/tmp
step() {  # name limit cmd...
  local name=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "$name rc=$rc: $(tail -c 300 "$OUT/$name.log" | tr '\n' ' ')"
  [ $rc -eq 0 ] || exit $rc
}
STAGES=${STAGES:-tests,smoke,bench,prof,hbm,fm,remote}
[[ $STAGES == *tests* ]] && step pytest_gpu 900 python -u -m pytest tests -m gpu -x -q --timeout 120 \
  --timeout-method thread -p no:cacheprovider
[[ $STAGES == *smoke* ]] && step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
[[ $STAGES == *bench* ]] && step bench 600 python bench.py
[[ $STAGES == *prof* ]] && step bench_prof 600 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o run \
  --output-format csv -- python bench.py --steps 5 --warmup 2
[[ $STAGES == *hbm* ]] && {
  step libsvm_hbm 300 python bench.py --mode hbm --steps 10 --warmup 2
  step libfm_hbm 300 python bench.py --mode hbm --format libfm --steps 10 --warmup 2
  step csv_hbm 300 python bench.py --mode hbm --format csv --steps 10 --warmup 2
  step recordio_hbm 300 python bench.py --mode hbm --format recordio --steps 10 --warmup 2
  step hashed 300 python scripts/bench_hashed.py --sweep 256,1024
}
[[ $STAGES == *fm* ]] && step linear 400 python scripts/bench_linear.py
[[ $STAGES == *remote* ]] && step remote_tls 600 python scripts/bench_remote.py --tls --epochs 2 \
  --threads 16 --reader-threads 16,32
exit 0
