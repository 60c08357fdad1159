#!/bin/bash
# Price the HBM-resident LibSVM fill (k_tile_fill) by parts: kernel traces of
# bench.py --mode hbm in several configurations, summarised per replayed chunk
# (time per GiB of text for the fill, the count, and the whole pass).
#   default        count + scan prelaunched on a second stream beside the fill
#   alone          --no-prelaunch: every kernel alone on the GPU
#   nostore        alone, DMLC_FILL_EXP=1: the fill without its CSR stores
#   nodecode       alone, DMLC_FILL_EXP=2: the fill without its token decode
#   neither        alone, DMLC_FILL_EXP=3
#   onepass        --one-pass: look-back fill, no count kernel
# The DMLC_FILL_EXP experiments exist only in a pricing build of the kernels
# (production kernels hold no experiment flags):
#   make clean && make HIPFLAGS_EXTRA=-DDMLC_FILL_PRICING all
# usage (through gpurun): bash scripts/fill_pricing.sh OUTDIR [format]
set -o pipefail
root="${GRAFT_REPO_ROOT:-$(pwd)}"
out="$root/gpurun_out/$1"
fmt=${2:-libsvm}
mkdir -p "$out"
export TMPDIR=/tmp
run() {  # name env... -- bench args
  local name=$1
  shift
  (cd /tmp && env "$@" timeout -k 10 300 rocprofv3 --kernel-trace -d "$out/$name" -o run \
     --output-format csv -- python3 "$root/bench.py" --mode hbm --format "$fmt" --steps 3 --warmup 1 \
     $BENCH_ARGS > "$out/$name.log" 2>&1) || { echo "$name failed"; tail -5 "$out/$name.log"; return 1; }
}
BENCH_ARGS="" run default DMLC_FILL_EXP=0 &&
BENCH_ARGS="--no-prelaunch" run alone DMLC_FILL_EXP=0 &&
BENCH_ARGS="--no-prelaunch" run nostore DMLC_FILL_EXP=1 &&
BENCH_ARGS="--no-prelaunch" run nodecode DMLC_FILL_EXP=2 &&
BENCH_ARGS="--no-prelaunch" run neither DMLC_FILL_EXP=3 &&
BENCH_ARGS="--one-pass" run onepass DMLC_FILL_EXP=0 || exit 1
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
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    # replayed chunks: the fills of >= 256 MiB (64 MiB streaming chunks excluded)
    big = [r for r in rows if "k_tile_fill" in r["Kernel_Name"]
           and int(r["Grid_Size_X"]) // 64 * 8192 >= (256 << 20)]
    cnt = [r for r in rows if "k_tile_count" in r["Kernel_Name"]
           and int(r["Grid_Size_X"]) // 64 * 8192 >= (256 << 20)]
    gib = lambda rs: sum(int(r["Grid_Size_X"]) // 64 * 8192 for r in rs) / (1 << 30)
    dur = lambda rs: sum(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in rs) / 1e3
    ent = {"fill_us_per_GiB": round(dur(big) / max(gib(big), 1e-9), 1),
           "count_us_per_GiB": round(dur(cnt) / max(gib(cnt), 1e-9), 1) if cnt else None,
           "fill_calls": len(big)}
    try:
        line = [l for l in open(os.path.join(out, name + ".log")) if l.startswith("{")][-1]
        b = json.loads(line)
        ent["ms_per_step"] = b["ms_per_step"]
        ent["input_GBps"] = b["input_GBps"]
    except Exception:
        pass
    res[name] = ent
json.dump(res, open(os.path.join(out, "pricing.json"), "w"), indent=1)
for k, v in res.items():
    print(k, v)
PY
