#!/bin/bash
# Round-4 GPU session in three parts (a gpurun call is capped at 20 minutes):
#   A: GPU tests, then the headline and format / mode benches
#   B: shapes, kernel traces
#   C: counter passes
# Each step runs under its own time limit; a part stops at its first failure.
# usage (through gpurun): bash scripts/r04_session.sh OUTDIR A|B|C
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}" || exit 1
o=$1/$2  # each part in its own directory (gpu_check numbers its commands from 1)
case "$2" in
  A)
    bash scripts/gpu_check.sh "$o" "tests -m gpu" \
      "python bench.py --steps 20 --warmup 5" \
      "python bench.py --mode hbm --steps 10 --warmup 2" \
      "python bench.py --mode hbm --format libfm --steps 10 --warmup 2" \
      "python bench.py --mode hbm --format csv --steps 10 --warmup 2" \
      "python bench.py --mode hbm --format recordio --steps 10 --warmup 2" \
      "python bench.py --mode cache --steps 10 --warmup 2" \
      "python bench.py --shuffle-parts 4 --steps 10 --warmup 2" \
      "python bench.py --mode hbm --shuffle-parts 4 --steps 10 --warmup 2" \
      "python scripts/bench_hashed.py --sweep 128,256,512,1024,2048" \
      "python scripts/bench_linear.py"
    ;;
  B)
    bash scripts/gpu_check.sh "$o" "" \
      "bash scripts/prof_kernels.sh $o/prof_hashed scripts/bench_hashed.py --sweep 256,1024" \
      "bash scripts/prof_kernels.sh $o/prof_linear scripts/bench_linear.py" \
      "bash scripts/prof_kernels.sh $o/prof_hbm bench.py --mode hbm --steps 5 --warmup 2" \
      "bash scripts/bench_shapes.sh $o/shapes libsvm"
    ;;
  C)
    bash scripts/gpu_check.sh "$o" "" \
      "bash scripts/pmc_kernels.sh gpurun_out/$o/pmc_hashed python scripts/bench_hashed.py --sweep '' --steps 3" \
      "bash scripts/pmc_kernels.sh gpurun_out/$o/pmc_uniform python bench.py --mode hbm --steps 2 --warmup 1" \
      "bash scripts/pmc_kernels.sh gpurun_out/$o/pmc_mixed python bench.py --mode hbm --shape mixed --rows 40000000 --steps 2 --warmup 1" \
      "bash scripts/pmc_kernels.sh gpurun_out/$o/pmc_csv python bench.py --mode hbm --format csv --steps 2 --warmup 1"
    ;;
  *) echo "part must be A, B or C"; exit 2 ;;
esac
