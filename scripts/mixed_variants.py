#!/usr/bin/env python3
"""Decompose the mixed LibSVM shape's fill cost: a skewed base file and
variants that each add one ingredient of `--shape mixed` (src/synthetic.cc
TextRow) -- qid tokens, weights on labels, exponent values, 9-12 digit
fractions, valueless tokens -- parsed on the GPU (one process per variant,
for rocprofv3 --pmc).
usage: python scripts/mixed_variants.py DIR make            (write the files)
       python scripts/mixed_variants.py DIR parse VARIANT   (parse one, 3 passes)"""
import os
import random
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
VARIANTS = ["base", "qid", "weight", "exp", "longfrac", "valueless", "all"]


def transform(line, row, v, rng):
    toks = line.split(" ")
    lab, feats = toks[0], toks[1:]
    if v in ("weight", "all") and row % 13 == 0:
        lab += ":0.%06d" % rng.randrange(10 ** 6)
    out = [lab]
    if v in ("qid", "all") and row % 17 == 0:
        out.append("qid:%d" % (row // 16))
    for t in feats:
        idx, _, val = t.partition(":")
        r = rng.randrange(16)
        if v in ("exp", "all") and r in (10, 11):
            val = "%d.%03de-%d" % (1 + rng.randrange(9), rng.randrange(1000), 1 + rng.randrange(5))
        elif v in ("longfrac", "all") and r == 12:
            val = "0." + "".join(str(rng.randrange(10)) for _ in range(9 + rng.randrange(4)))
        elif v in ("valueless", "all") and r in (13, 14):
            out.append(idx)
            continue
        out.append(idx + ":" + val)
    return " ".join(out)


def main():
    d, cmd = sys.argv[1], sys.argv[2]
    from dmlc_core_amd import data
    if cmd == "make":
        os.makedirs(d, exist_ok=True)
        base = os.path.join(d, "base.libsvm")
        if not os.path.exists(base):
            data.write_synthetic(base, 0, 400000, format="libsvm", seed=7, nthread=8, shape="skewed")
        lines = open(base).read().splitlines()
        for v in VARIANTS[1:]:
            rng = random.Random(v)
            with open(os.path.join(d, v + ".libsvm"), "w") as f:
                for i, ln in enumerate(lines):
                    f.write(transform(ln, i, v, rng) + "\n")
        return
    import torch
    p = os.path.join(d, sys.argv[3] + ".libsvm")
    g = data.GPUParser(p)
    for _ in range(3):
        g.before_first()
        csr = g.parse_all()
    torch.cuda.synchronize()
    print(sys.argv[3], csr.rows, g.stats().get("exact_chunks"), os.path.getsize(p))


if __name__ == "__main__":
    main()
