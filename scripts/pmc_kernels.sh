#!/bin/bash
# PMC counters (three passes, one counter group each) of any python command,
# summarised per kernel into OUT/pmc_summary.json.
# usage (through gpurun): bash scripts/pmc_kernels.sh OUT python script.py args...
set -o pipefail
OUT=$1; shift
mkdir -p "$OUT"
export TMPDIR=/tmp
P1="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY"
P2="SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS"
P3="FETCH_SIZE GRBM_GUI_ACTIVE GRBM_COUNT"
P4="WRITE_SIZE"
i=0
for P in "$P1" "$P2" "$P3" "$P4"; do
  i=$((i+1))
  timeout -s KILL 150 rocprofv3 --pmc $P -d "$OUT/p$i" -o run --output-format csv -- "$@" \
    > "$OUT/p$i.log" 2>&1 || { echo "pass $i failed"; tail -5 "$OUT/p$i.log"; exit 1; }
done
python - "$OUT" <<'PY'
import csv, glob, sys, collections, json, re
out = sys.argv[1]
agg = collections.defaultdict(lambda: collections.defaultdict(float))
cnt = collections.defaultdict(set)
for f in glob.glob(f"{out}/p*/**/*counter_collection.csv", recursive=True):
    for row in csv.DictReader(open(f)):
        m = re.search(r"(k_\w+)(<[^(]*>)?", row["Kernel_Name"])
        k = (m.group(1) + (m.group(2) or "")) if m else row["Kernel_Name"][:40]
        agg[k][row["Counter_Name"]] += float(row["Counter_Value"])
        cnt[k].add(row.get("Dispatch_Id", row.get("Correlation_Id", "")))
res = {k: dict(v, dispatches=len(cnt[k])) for k, v in agg.items()}
json.dump(res, open(f"{out}/pmc_summary.json", "w"), indent=1)
for k, v in res.items():
    if k.startswith("k_"):
        print(k, {a: round(b) for a, b in v.items()})
PY
