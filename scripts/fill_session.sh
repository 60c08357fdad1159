#!/bin/bash
# Text-fill measurement session: HBM-resident LibSVM / LibFM epochs, the
# hashed fp8 sweep, then rocprofv3 VALU counters of the tile kernels.
# Every GPU step has its own timeout; a failure ends the script.
#   OUT=gpurun_out/fill TAG=base bash scripts/fill_session.sh
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=${OUT:-gpurun_out/fill}
TAG=${TAG:-run}
STAGES=${STAGES:-bench,hashed,pmc}
mkdir -p "$OUT"
export TMPDIR=/tmp
run() {  # name timeout cmd...
  local name=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > "$OUT/${TAG}_$name.json" 2> "$OUT/${TAG}_$name.err"
  local rc=$?
  echo "$name rc=$rc $(tail -c 600 "$OUT/${TAG}_$name.json")"
  [ $rc -eq 0 ] || { tail -5 "$OUT/${TAG}_$name.err"; exit $rc; }
}
if [[ $STAGES == *bench* ]]; then
  run libsvm_hbm 300 python bench.py --mode hbm --steps 10 --warmup 2
  run libfm_hbm 300 python bench.py --mode hbm --format libfm --steps 10 --warmup 2
fi
if [[ $STAGES == *csv* ]]; then
  run csv_hbm 300 python bench.py --mode hbm --format csv --steps 10 --warmup 2
fi
if [[ $STAGES == *hashed* ]]; then
  run hashed 300 python scripts/bench_hashed.py --sweep 256,1024
fi
if [[ $STAGES == *pmc* ]]; then
  for fmt in libsvm libfm ${PMC_EXTRA:-}; do
    timeout -s KILL 180 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES \
      -d "$OUT/pmc_${TAG}_$fmt" -o run --output-format csv -- \
      python3 bench.py --rows 2000000 --mode hbm --format $fmt --steps 3 --warmup 1 > "$OUT/pmc_${TAG}_$fmt.log" 2>&1
    rc=$?; echo "pmc $fmt rc=$rc"
    [ $rc -eq 0 ] || { tail -5 "$OUT/pmc_${TAG}_$fmt.log"; exit $rc; }
  done
  timeout -s KILL 180 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES \
    -d "$OUT/pmc_${TAG}_hashed" -o run --output-format csv -- \
    python3 scripts/bench_hashed.py --sweep 1024 --steps 2 > "$OUT/pmc_${TAG}_hashed.log" 2>&1
  rc=$?; echo "pmc hashed rc=$rc"
  [ $rc -eq 0 ] || { tail -5 "$OUT/pmc_${TAG}_hashed.log"; exit $rc; }
  python3 scripts/pmc_per_wave.py "$OUT" "$TAG"
fi
exit 0
