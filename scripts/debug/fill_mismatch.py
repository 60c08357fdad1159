"""Debug helper: GPU tile fill vs CPU parser, print the first mismatching rows."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import numpy as np
from dmlc_core_amd import data

p = "/tmp/dbg.libsvm"
rows = int(sys.argv[1]) if len(sys.argv) > 1 else 30000
chunk = int(sys.argv[2]) if len(sys.argv) > 2 else (1 << 20)
data.write_synthetic(p, 0, rows, seed=5)
h = data.GPUParser(p, chunk_bytes=chunk, zero_copy=0).parse_all().to_host()
cpu = list(data.iter_blocks(p))
lab = np.concatenate([b["label"] for b in cpu])
off = np.concatenate([[0], np.cumsum([len(b["index"]) for b in cpu])])
cnt = np.concatenate([np.diff(b["offset"]) for b in cpu])
coff = np.concatenate([[0], np.cumsum(cnt)])
idx = np.concatenate([b["index"] for b in cpu])
val = np.concatenate([b["value"] for b in cpu])
print("rows", len(lab), h["label"].shape, "nnz", len(idx), h["index"].shape)
bad = np.nonzero(h["label"] != lab)[0]
print("label mismatches", len(bad), bad[:20])
text = open(p, "rb").read()
starts = [0] + [i + 1 for i, c in enumerate(text) if c == 10][:-1]
for r in bad[:6]:
    s = starts[r]
    print(r, "byte", s, "tile", s // 8192, "in-tile", s % 8192, "gpu", h["label"][r], "cpu", lab[r],
          repr(text[max(0, s - 20):s + 30]))
ob = np.nonzero(h["offset"] != coff)[0]
print("offset mismatches", len(ob), ob[:10])
ib = np.nonzero(h["index"] != idx)[0] if len(h["index"]) == len(idx) else []
print("index mismatches", len(ib), ib[:10])
vb = np.nonzero(h["value"] != val)[0] if len(h["value"]) == len(val) else []
print("value mismatches", len(vb), vb[:10])
for j in vb[:5]:
    print(j, h["value"][j], val[j], h["index"][j], idx[j])
print("---- offset mismatch context")
for r in ob[:8]:
    s = starts[r]
    print(r, "byte", s, "tile", s // 8192, "in-tile", s % 8192, "step", (s % 8192) // 2048,
          "gpu off", h["offset"][r], "cpu off", coff[r], "gpu lab", h["label"][r], "cpu lab", lab[r])
if len(ob):
    r = ob[0]
    print(repr(text[starts[r - 1]:starts[r + 2]]))
ok = not (len(bad) or len(ob) or len(ib) or len(vb))
print("PARITY", "OK" if ok else "FAILED")
sys.exit(0 if ok else 1)
