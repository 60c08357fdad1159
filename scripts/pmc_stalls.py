"""Per-wave averages of every counter in rocprofv3 --pmc CSVs, per tile kernel.
usage: python scripts/pmc_stalls.py DIR [DIR ...]  (prints one line per kernel)"""
import collections
import csv
import glob
import re
import sys

for d in sys.argv[1:]:
    agg = collections.defaultdict(lambda: collections.defaultdict(float))
    for f in glob.glob(f"{d}/**/*counter_collection.csv", recursive=True):
        for row in csv.DictReader(open(f)):
            m = re.search(r"(k_\w+)(<.*?>)?(?=\()", row["Kernel_Name"])  # (template args kept)
            k = (m.group(1) + (m.group(2) or "")) if m else row["Kernel_Name"][:40]
            agg[k][row["Counter_Name"]] += float(row["Counter_Value"])
    for k, v in sorted(agg.items()):
        w = v.get("SQ_WAVES", 0)
        if w > 1000:
            print(d.rstrip("/").rsplit("/", 1)[-1], k, {c: round(x / w, 1) for c, x in v.items()})
