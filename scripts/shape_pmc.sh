#!/usr/bin/env bash
# VALU / SALU per tile of the tile kernels on the realistic LibSVM shapes
# (HBM-resident epochs), summarised by scripts/pmc_per_wave.py.
#   OUT=gpurun_out/shape_pmc TAG=x bash scripts/shape_pmc.sh
set -u
OUT=${OUT:-gpurun_out/shape_pmc}
TAG=${TAG:-shapes}
mkdir -p "$OUT"
export TMPDIR=/tmp
for shape in ${SHAPES:-skewed mixed}; do
  timeout -s KILL 240 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES \
    -d "$OUT/pmc_${TAG}_$shape" -o run --output-format csv -- \
    python3 bench.py --rows 8000000 --shape $shape --mode hbm --steps 3 --warmup 1 > "$OUT/pmc_${TAG}_$shape.log" 2>&1
  rc=$?; echo "pmc $shape rc=$rc"
  [ $rc -eq 0 ] || { tail -5 "$OUT/pmc_${TAG}_$shape.log"; exit $rc; }
done
python3 scripts/pmc_per_wave.py "$OUT" "$TAG"
