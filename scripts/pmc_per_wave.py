"""Per-wave VALU / SALU of the tile kernels from rocprofv3 --pmc CSVs
(one wave = one 8 KiB tile for k_tile_count / k_tile_fill / k_tile_hash).
usage: python scripts/pmc_per_wave.py OUT_DIR TAG  -> OUT_DIR/pmc_TAG.json"""
import collections
import csv
import glob
import json
import re
import sys

out, tag = sys.argv[1], sys.argv[2]
res = {}
for d in sorted(glob.glob(f"{out}/pmc_{tag}_*/")):
    name = d.rstrip("/").rsplit("_", 1)[1]
    agg = collections.defaultdict(lambda: collections.defaultdict(float))
    for f in glob.glob(f"{d}/**/*counter_collection.csv", recursive=True):
        for row in csv.DictReader(open(f)):
            m = re.search(r"(k_\w+)(<.*?>)?(?=\()", row["Kernel_Name"])  # (template args kept)
            k = (m.group(1) + (m.group(2) or "")) if m else row["Kernel_Name"][:40]
            agg[k][row["Counter_Name"]] += float(row["Counter_Value"])
    per = {}
    for k, v in agg.items():
        if v.get("SQ_WAVES", 0) > 0 and "tile" in k:
            w = v["SQ_WAVES"]
            per[k] = {"waves": int(w), "valu_per_wave": round(v.get("SQ_INSTS_VALU", 0) / w, 1),
                      "salu_per_wave": round(v.get("SQ_INSTS_SALU", 0) / w, 1),
                      "wave_cycles_per_wave": round(v.get("SQ_WAVE_CYCLES", 0) / w, 1)}
    res[name] = per
json.dump(res, open(f"{out}/pmc_{tag}.json", "w"), indent=1)
for name, per in res.items():
    for k, v in per.items():
        print(name, k, v)
