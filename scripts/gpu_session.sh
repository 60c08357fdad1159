#!/bin/bash
# One GPU session: gpu tests -> bench -> rocprofv3 kernel stats.
# Every GPU step has its own timeout; a fault / abort / timeout ends the script.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
OUT=gpurun_out
export TMPDIR=/tmp
STAGES="${STAGES:-test,bench,prof}"
BENCH_ARGS="${BENCH_ARGS:---steps 5 --warmup 2}"
echo "== host: $(nproc) cpus"; df -h /tmp | tail -1; free -g | head -2
rocm-smi --showproductname 2>/dev/null | grep -E 'GPU|Card' | head -3 || true
ok() { local rc=$1; [ "$rc" -eq 0 ] || [ "$rc" -eq 1 ]; }
if [[ $STAGES == *test* ]]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -p no:cacheprovider > $OUT/pytest_gpu.log 2>&1
  rc=$?; echo "pytest gpu rc=$rc"; tail -25 $OUT/pytest_gpu.log
  ok $rc || exit $rc
fi
if [[ $STAGES == *h2d* ]]; then
  timeout -k 10 300 python scripts/h2d_bw.py > $OUT/h2d.json 2>&1; echo "h2d rc=$?"; cat $OUT/h2d.json
fi
if [[ $STAGES == *bench* ]]; then
  timeout -k 10 900 python bench.py $BENCH_ARGS > $OUT/bench.json 2> $OUT/bench.err
  rc=$?; echo "bench rc=$rc"; cat $OUT/bench.json; tail -5 $OUT/bench.err
  [ $rc -eq 0 ] || exit $rc
  if [ -n "${BENCH2_ARGS:-}" ]; then
    timeout -k 10 900 python bench.py $BENCH2_ARGS > $OUT/bench2.json 2> $OUT/bench2.err
    rc=$?; echo "bench2 rc=$rc"; cat $OUT/bench2.json; tail -5 $OUT/bench2.err
    [ $rc -eq 0 ] || exit $rc
  fi
fi
if [[ $STAGES == *prof* ]]; then
  timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- \
    python3 bench.py --steps 2 --warmup 1 > $OUT/prof_bench.log 2>&1
  rc=$?; echo "rocprof rc=$rc"; tail -3 $OUT/prof_bench.log
  find $OUT/prof -name '*kernel_stats*' | head -3
fi
exit 0
