"""Pure-Python reference of the framework's text grammars (documented in
src/data/libsvm_parser.h, libfm_parser.h, csv_parser.h) and of the reference
dmlc strtof arithmetic, used as an independent oracle for the C++ and HIP
parsers."""
import struct

import numpy as np

DIGITCHARS = set("0123456789+-.eE")


def f32(x):
    return struct.unpack("f", struct.pack("f", x))[0]


def strtof(s: str) -> float:
    """Reference dmlc::data::strtof arithmetic (src/data/strtonum.h:37-97)."""
    p, n = 0, len(s)
    sign = True
    if p < n and s[p] == "-":
        sign, p = False, p + 1
    elif p < n and s[p] == "+":
        p += 1
    value = f32(0.0)
    while p < n and s[p].isdigit():
        value = f32(f32(value * f32(10.0)) + f32(float(ord(s[p]) - 48)))
        p += 1
    if p < n and s[p] == ".":
        p += 1
        pow10, val2 = 1, 0
        while p < n and s[p].isdigit():
            val2 = (val2 * 10 + ord(s[p]) - 48) % (1 << 64)
            pow10 = (pow10 * 10) % (1 << 64)
            p += 1
        value = f32(value + f32(float(val2) / float(pow10)))
    if p < n and s[p] in "eE":
        p += 1
        frac = False
        if p < n and s[p] == "-":
            frac, p = True, p + 1
        elif p < n and s[p] == "+":
            p += 1
        expon = 0
        while p < n and s[p].isdigit():
            expon = (expon * 10 + ord(s[p]) - 48) % (1 << 32)
            p += 1
        expon = min(expon, 38)
        scale = f32(1.0)
        while expon >= 8:
            scale = f32(scale * 1e8)
            expon -= 8
        while expon > 0:
            scale = f32(scale * 10.0)
            expon -= 1
        value = f32(value / scale) if frac else f32(value * scale)
    return value if sign else -value


def strtouint(s: str, bits: int = 32) -> int:
    p = 0
    if p < len(s) and s[p] in "+-":
        p += 1
    v = 0
    while p < len(s) and s[p].isdigit():
        v = (v * 10 + ord(s[p]) - 48) % (1 << bits)
        p += 1
    return v


def parse_pair(tok: str, t1, t2):
    """ParsePair inside one token -> (r, v1, v2)."""
    i, n = 0, len(tok)
    while i < n and tok[i] not in DIGITCHARS:
        i += 1
    if i == n:
        return 0, None, None
    j = i
    while j < n and tok[j] in DIGITCHARS:
        j += 1
    v1 = t1(tok[i:j])
    p = j
    while p < n and tok[p] in " \t":
        p += 1
    if p == n or tok[p] != ":":
        return 1, v1, None
    p += 1
    while p < n and tok[p] not in DIGITCHARS:
        p += 1
    q = p
    while q < n and tok[q] in DIGITCHARS:
        q += 1
    return 2, v1, t2(tok[p:q])


def parse_triple(tok: str):
    r, a, rest = 0, None, None
    i, n = 0, len(tok)
    while i < n and tok[i] not in DIGITCHARS:
        i += 1
    if i == n:
        return 0, None, None, None
    j = i
    while j < n and tok[j] in DIGITCHARS:
        j += 1
    a = strtouint(tok[i:j])
    if j == n or tok[j] != ":":
        return 1, a, None, None
    r2, b, c = parse_pair(tok[j + 1:], strtouint, strtof)
    if r2 == 0:
        return 2, a, 0, None
    if r2 == 1:
        return 2, a, b, None
    return 3, a, b, c


def _lines(text: str):
    import re
    for line in re.split(r"[\r\n]+", text):
        if line:
            yield line


def parse_libsvm(text: str):
    rows = []  # (label, weight|None, qid|None, [(idx, val|None)])
    for line in _lines(text):
        toks = [t for t in line.replace("\t", " ").split(" ") if t]
        if not toks:
            continue
        r, lab, w = parse_pair(toks[0], strtof, strtof)
        if r < 1:
            continue
        qid = None
        feats = []
        for k, tok in enumerate(toks[1:]):
            if k == 0 and tok.startswith("qid:"):
                s = tok[4:]
                neg = s.startswith("-")
                v = strtouint(s.lstrip("+-"), 64)
                qid = (-v) % (1 << 64) if neg else v
                continue
            rr, idx, val = parse_pair(tok, strtouint, strtof)
            if rr < 1:
                continue
            feats.append((idx, val if rr == 2 else None))
        rows.append((lab, w if r == 2 else None, qid, feats))
    return rows


def parse_libfm(text: str):
    rows = []
    for line in _lines(text):
        toks = [t for t in line.replace("\t", " ").split(" ") if t]
        if not toks:
            continue
        r, lab, w = parse_pair(toks[0], strtof, strtof)
        if r < 1:
            continue
        feats = []
        for tok in toks[1:]:
            rr, fid, idx, val = parse_triple(tok)
            if rr <= 1:
                continue
            feats.append((fid, idx, val if rr == 3 else None))
        rows.append((lab, w if r == 2 else None, feats))
    return rows


def parse_csv(text: str, label_column=-1, delim=","):
    rows = []
    for line in _lines(text):
        fields = line.split(delim)
        # reference csv_parser.h:83-96: after skipping a delimiter the loop stops
        # when p reaches the line end, so a trailing delimiter adds no field
        if len(fields) > 1 and fields[-1] == "":
            fields.pop()
        lab = 0.0
        feats = []
        for c, f in enumerate(fields):
            v = strtof(f.lstrip(" \t\r\n\f"))
            if c == label_column:
                lab = v
            else:
                feats.append(v)
        rows.append((lab, feats))
    return rows


def concat_blocks(blocks):
    """Concatenate host blocks into semantic per-row arrays (NULL -> default)."""
    label, weight, qid, offset, index, value, field = [], [], [], [0], [], [], []
    for b in blocks:
        n = len(b["label"])
        label.append(b["label"])
        weight.append(b["weight"] if b["weight"] is not None else np.ones(n, np.float32))
        qid.append(b["qid"] if b["qid"] is not None else np.zeros(n, np.uint64))
        nnz = len(b["index"])
        index.append(b["index"])
        value.append(b["value"] if b["value"] is not None else np.ones(nnz, np.float32))
        if b.get("field") is not None:
            field.append(b["field"])
        offset.extend((b["offset"][1:] + offset[-1]).tolist())
    cat = lambda xs, dt: np.concatenate(xs).astype(dt) if xs else np.zeros(0, dt)  # noqa: E731
    return {
        "label": cat(label, np.float32), "weight": cat(weight, np.float32),
        "qid": cat(qid, np.uint64), "offset": np.array(offset, np.uint64),
        "index": cat(index, np.uint64), "value": cat(value, np.float32),
        "field": cat(field, np.uint64) if field else None,
    }
