#!/bin/bash
# r05 session 9: persistent RecordIO fill with the next tile prefetched
# (DMLC_REC_FILL_PF 0 = a wave per tile, 1 = loads issued after staging,
# 2 = after the header walk).
out=gpurun_out/r05_s9
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
PYT="python -u -m pytest -x -v --timeout 150 --timeout-method thread"
step pytest_rec 400 $PYT tests/test_gpu_recordio.py
DMLC_REC_FILL_PF=1 step pytest_rec_pf1 400 $PYT tests/test_gpu_recordio.py
for pf in 0 1 2; do
  DMLC_REC_FILL_PF=$pf step bench_pf$pf 300 python -u bench.py --mode hbm --format recordio --steps 10 --warmup 2
done
for pf in 1 2; do
  DMLC_REC_FILL_PF=$pf step prof_pf$pf 400 bash -c "cd /tmp && rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$out/prof_pf$pf -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --mode hbm --format recordio --steps 5 --warmup 2"
done
