#!/bin/bash
# Price the HBM-resident CSV fill (k_csv_tile_fill) by parts: kernel traces of
# bench.py --mode hbm --format csv, each kernel alone on the GPU
# (--no-prelaunch), summarised as time per GiB of text of the replayed chunks.
#   alone     production kernel
#   nodecode  DMLC_CSV_EXP=1: fields listed, no number decode
#   nostore   DMLC_CSV_EXP=2: decoded, no CSR stores
#   neither   DMLC_CSV_EXP=3
#   norounds  DMLC_CSV_EXP=4: masks, scans and listing only
# usage (through gpurun): bash scripts/csv_pricing.sh OUTDIR
set -o pipefail
root="${GRAFT_REPO_ROOT:-$(pwd)}"
out="$root/gpurun_out/$1"
mkdir -p "$out"
export TMPDIR=/tmp
run() {  # name exp
  (cd /tmp && DMLC_CSV_EXP=$2 timeout -k 10 300 rocprofv3 --kernel-trace -d "$out/$1" -o run \
     --output-format csv -- python3 "$root/bench.py" --mode hbm --format csv --steps 3 --warmup 1 \
     --no-prelaunch > "$out/$1.log" 2>&1) || { echo "$1 failed"; tail -5 "$out/$1.log"; return 1; }
}
run alone 0 && run nodecode 1 && run nostore 2 && run neither 3 && run norounds 4 || exit 1
python3 - "$out" <<'PY'
import csv, glob, json, os, sys
out = sys.argv[1]
res = {}
for d in sorted(glob.glob(os.path.join(out, "*/"))):
    name = os.path.basename(d.rstrip("/"))
    f = glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True)
    if not f:
        continue
    rows = list(csv.DictReader(open(f[0])))
    def pick(k):
        return [r for r in rows if k in r["Kernel_Name"]
                and int(r["Grid_Size_X"]) // 64 * 8192 >= (256 << 20)]
    gib = lambda rs: sum(int(r["Grid_Size_X"]) // 64 * 8192 for r in rs) / (1 << 30)
    dur = lambda rs: sum(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in rs) / 1e3
    fill, cnt = pick("k_csv_tile_fill"), pick("k_csv_tile_count")
    res[name] = {"fill_us_per_GiB": round(dur(fill) / max(gib(fill), 1e-9), 1),
                 "count_us_per_GiB": round(dur(cnt) / max(gib(cnt), 1e-9), 1), "calls": len(fill)}
json.dump(res, open(os.path.join(out, "pricing.json"), "w"), indent=1)
for k, v in res.items():
    print(k, v)
PY
