#!/usr/bin/env bash
# VALU per tile of the fill on skewed LibSVM plus one mixed-shape ingredient
# at a time (scripts/mixed_variants.py), one rocprofv3 --pmc pass per variant.
set -u
OUT=${OUT:-gpurun_out/mixed_variants}
D=${D:-/tmp/dmlc_mixed_variants}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 300 python3 scripts/mixed_variants.py "$D" make || exit 1
for v in ${VARIANTS:-base qid weight exp longfrac valueless all}; do
  timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES \
    -d "$OUT/pmc_mv_$v" -o run --output-format csv -- python3 scripts/mixed_variants.py "$D" parse $v \
    > "$OUT/pmc_mv_$v.log" 2>&1
  rc=$?; echo "pmc $v rc=$rc $(tail -1 "$OUT/pmc_mv_$v.log")"
  [ $rc -eq 0 ] || exit $rc
done
python3 scripts/pmc_per_wave.py "$OUT" mv | grep -E "k_tile_(fill|count)"
