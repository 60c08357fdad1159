#!/bin/bash
# rocprofv3 --kernel-trace --stats of one python command; the summary CSV lands
# in gpurun_out/OUTDIR/.  usage: scripts/prof_kernels.sh OUTDIR script.py [args...]
set -o pipefail
root="${GRAFT_REPO_ROOT:-$(pwd)}"
out="$root/gpurun_out/$1"; shift
mkdir -p "$out"
export TMPDIR=/tmp
cd /tmp || exit 1
timeout -k 10 500 rocprofv3 --kernel-trace --stats -d "$out" -o run --output-format csv \
  -- python3 "$root/$@" > "$out/run.log" 2>&1
rc=$?
tail -3 "$out/run.log"
f=$(find "$out" -name '*kernel_stats.csv' | head -1)
[ -n "$f" ] && python3 - "$f" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: -float(r["TotalDurationNs"]))
for r in rows[:14]:
    print("%-60s calls %6s avg %10.1f us  total %10.1f ms" % (r["Name"][:60], r["Calls"],
          float(r["AverageNs"]) / 1e3, float(r["TotalDurationNs"]) / 1e6))
PY
exit $rc
