"""Compare the GPU tile parse of a synthetic LibSVM / LibFM file with the CPU
parser and print the first mismatching entries with their text (debug aid)."""
import sys

import numpy as np

sys.path.insert(0, ".")
from dmlc_core_amd import data  # noqa: E402

fmt = sys.argv[1] if len(sys.argv) > 1 else "libsvm"
rows = int(sys.argv[2]) if len(sys.argv) > 2 else 20000
p = f"/tmp/dbg.{fmt}"
data.write_synthetic(p, 0, rows, format=fmt, seed=5)
g = data.GPUParser(p, format=fmt).parse_all().to_host()
cpu = list(data.iter_blocks(p, 0, 1, fmt))
idx = np.concatenate([b["index"] for b in cpu])
val = np.concatenate([b["value"] for b in cpu])
lab = np.concatenate([b["label"] for b in cpu])
off = np.cumsum([0] + [len(b["index"]) for b in cpu for _ in [0]])
print("rows", len(lab), len(g["label"]), "nnz", len(idx), len(g["index"]))
print("label eq", np.array_equal(lab, g["label"]))
n = min(len(idx), len(g["index"]))
bad = np.nonzero((idx[:n] != g["index"][:n]) | (val[:n] != g["value"][:n]))[0]
print("mismatches", len(bad))
text = open(p, "rb").read()
toks = [t for line in text.split(b"\n") for t in line.split(b" ")[1:] if t]
for k in bad[:20]:
    print(k, "cpu", idx[k], val[k], "gpu", g["index"][k], g["value"][k],
          "text", toks[k] if k < len(toks) else None)
