#!/bin/bash
# GPU-box validation driver (run through gpurun): pytest selection, then
# optional extra commands, each under its own time limit; stops at the first
# failure.  usage: scripts/gpu_check.sh OUTDIR "PYTEST_ARGS" ["CMD" ...]
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}" || exit 1
out=gpurun_out/$1; shift
mkdir -p "$out"
export TMPDIR=/tmp
if [ -n "$1" ]; then
  timeout -k 10 900 python -u -m pytest $1 -q --timeout 120 --timeout-method thread \
    -p no:cacheprovider > "$out/pytest.log" 2>&1
  rc=$?
  tail -3 "$out/pytest.log"
  [ $rc -eq 0 ] || exit $rc
fi
shift
i=0
for cmd in "$@"; do
  i=$((i + 1))
  timeout -k 10 600 bash -c "$cmd" > "$out/cmd$i.out" 2> "$out/cmd$i.err"
  rc=$?
  echo "cmd$i rc=$rc: $cmd"
  tail -c 2000 "$out/cmd$i.out"
  [ $rc -eq 0 ] || { tail -20 "$out/cmd$i.err"; exit $rc; }
done
