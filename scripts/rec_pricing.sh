#!/bin/bash
# Price the HBM-resident RecordIO decode: bench.py --mode hbm --format recordio
# under kernel traces -- counted path (default), one pass, and one-pass
# ablations (DMLC_REC_EXP: 1 no look-back wait, 2 no payload copies).
# usage (through gpurun): bash scripts/rec_pricing.sh OUTDIR
set -o pipefail
root="${GRAFT_REPO_ROOT:-$(pwd)}"
out="$root/gpurun_out/$1"
mkdir -p "$out"
export TMPDIR=/tmp
run() {  # name exp args...
  local name=$1 exp=$2
  shift 2
  (cd /tmp && DMLC_REC_EXP=$exp timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$out/$name" -o run \
     --output-format csv -- python3 "$root/bench.py" --mode hbm --format recordio --steps 5 --warmup 1 \
     "$@" > "$out/$name.log" 2>&1) || { echo "$name failed"; tail -5 "$out/$name.log"; return 1; }
  f=$(find "$out/$name" -name '*kernel_stats.csv' | head -1)
  echo "== $name: $(grep -o '"ms_per_step": [0-9.]*' "$out/$name.log")"
  python3 - "$f" <<'PY'
import csv, sys
for r in sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: -float(r["TotalDurationNs"]))[:5]:
    print("   %-50s calls %4s avg %9.1f us" % (r["Name"][:50], r["Calls"], float(r["AverageNs"]) / 1e3))
PY
}
run onepass 0 --one-pass && run counted 0 && run nolookback 1 --one-pass && run nocopy 2 --one-pass && run neither 3 --one-pass
