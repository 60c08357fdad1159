#!/usr/bin/env python3
"""Per-kernel averages of rocprofv3 --pmc counter CSVs (one row per dispatch x counter).

usage: python scripts/pmc_summary.py gpurun_out/pmc1 gpurun_out/pmc2 ... [--json out.json]
"""
import collections
import csv
import glob
import json
import os
import re
import sys


def kernel_key(name: str) -> str:
    m = re.search(r"(k_\w+)", name)
    if m:
        fmt = re.search(r"TextFormat\)(\d)", name)
        return m.group(1) + (f"<fmt{fmt.group(1)}>" if fmt else "")
    return name[:40]


def summarize(dirs):
    agg = collections.defaultdict(lambda: collections.defaultdict(float))
    disp = collections.defaultdict(lambda: collections.defaultdict(set))
    for d in dirs:
        for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
            for r in csv.DictReader(open(f)):
                k = kernel_key(r["Kernel_Name"])
                c = r["Counter_Name"]
                agg[k][c] += float(r["Counter_Value"])
                disp[k][c].add((f, r["Dispatch_Id"]))
    out = {}
    for k, v in agg.items():
        out[k] = {c: round(x / max(1, len(disp[k][c])), 1) for c, x in v.items()}
        out[k]["dispatches"] = max(len(s) for s in disp[k].values())
    return out


if __name__ == "__main__":
    args = [a for a in sys.argv[1:] if not a.startswith("--")]
    res = summarize(args)
    for k, v in sorted(res.items()):
        print(k, json.dumps(v))
    if "--json" in sys.argv:
        with open(sys.argv[sys.argv.index("--json") + 1], "w") as f:
            json.dump(res, f, indent=1)
