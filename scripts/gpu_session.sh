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
if [[ $STAGES == *hashed* ]]; then
  timeout -k 10 600 python scripts/bench_hashed.py ${HASHED_ARGS:-} > $OUT/hashed.json 2> $OUT/hashed.err
  rc=$?; echo "hashed rc=$rc"; cat $OUT/hashed.json; tail -5 $OUT/hashed.err
  [ $rc -eq 0 ] || exit $rc
  timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $OUT/prof_hashed -o run --output-format csv -- \
    python3 scripts/bench_hashed.py --steps 1 ${HASHED_ARGS:-} > $OUT/prof_hashed.log 2>&1
  rc=$?; echo "rocprof hashed rc=$rc"
  [ $rc -eq 0 ] || exit $rc
fi
PROF_ARGS="${PROF_ARGS:---steps 2 --warmup 1}"
if [[ $STAGES == *prof* ]]; then
  timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- \
    python3 bench.py $PROF_ARGS > $OUT/prof_bench.log 2>&1
  rc=$?; echo "rocprof rc=$rc"; tail -3 $OUT/prof_bench.log
  find $OUT/prof -name '*kernel_stats*' | head -3
  [ $rc -eq 0 ] || exit $rc
fi
# hardware counters: one rocprofv3 pass per counter group (slot limits:
# FETCH_SIZE and WRITE_SIZE each need their own pass), counters only
PMC_ARGS="${PMC_ARGS:---rows 2000000 --mode hbm --steps 3 --warmup 1}"
if [[ $STAGES == *pmc* ]]; then
  i=0
  for grp in "FETCH_SIZE" "WRITE_SIZE" \
             "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAVE_CYCLES SQ_BUSY_CYCLES"; do
    i=$((i+1))
    timeout -s KILL 240 rocprofv3 --pmc $grp -d $OUT/pmc$i -o run --output-format csv -- \
      python3 bench.py $PMC_ARGS > $OUT/pmc$i.log 2>&1
    rc=$?; echo "pmc pass $i ($grp) rc=$rc"; tail -2 $OUT/pmc$i.log
    case $rc in 0|1|2) ;; *) exit $rc ;; esac
  done
fi
exit 0
