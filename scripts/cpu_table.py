"""Best-of table of scripts/cpu_baseline.sh results (ref vs repo per dataset
and thread count).  usage: python scripts/cpu_table.py cpu.jsonl"""
import collections
import json
import sys

best = collections.defaultdict(float)
for line in open(sys.argv[1]):
    line = line.strip()
    if not line.startswith("{"):
        continue
    d = json.loads(line)
    r = d["result"]
    uri = r["uri"].split("/")[-1].split("?")[0]
    mode = r.get("mode") or r.get("format")
    key = (f"{uri} {mode}", d["omp_threads"], d["impl"])
    rate = r.get("rows_per_sec") or r.get("records_per_sec")
    best[key] = max(best[key], rate)
rows = sorted({(k[0], k[1]) for k in best})
print("| dataset | threads | ref M/s | repo M/s | repo / ref |")
print("|---|---|---|---|---|")
for ds, t in rows:
    a, b = best[(ds, t, "ref")], best[(ds, t, "repo")]
    print(f"| {ds} | {t} | {a / 1e6:.2f} | {b / 1e6:.2f} | {b / a if a else 0:.2f}x |")
