"""Static instruction count per source line of one kernel (hipcc -g -S listing).
usage: python scripts/asm_lines.py file.s <kernel-substring> [top]"""
import collections
import re
import sys

s = open(sys.argv[1]).read().splitlines()
start = next(i for i, l in enumerate(s) if re.match(r"^_Z\S*" + re.escape(sys.argv[2]) + r"\S*:", l))
end = next(i for i in range(start, len(s)) if s[i].startswith(".Lfunc_end"))
files = {}
for l in s:
    m = re.match(r'\s*\.file\s+(\d+)\s+"([^"]*)"(?:\s+"([^"]*)")?', l)
    if m:
        files[m.group(1)] = (m.group(3) or m.group(2)).split("/")[-1]
cur = "?"
tot = collections.Counter()
kinds = collections.defaultdict(collections.Counter)
for l in s[start:end]:
    m = re.match(r"\s*\.loc\s+(\d+)\s+(\d+)", l)
    if m:
        cur = files.get(m.group(1), "?") + ":" + m.group(2)
        continue
    t = l.strip()
    if l.startswith("\t") and not t.startswith((".", ";")):
        op = t.split()[0]
        k = ("V" if op.startswith("v_") else "S" if op.startswith("s_")
             else "D" if op.startswith("ds_") else "M")
        tot[cur] += 1
        kinds[cur][k] += 1
src = {}
for line, n in tot.most_common(int(sys.argv[3]) if len(sys.argv) > 3 else 40):
    f, ln = line.rsplit(":", 1)
    text = ""
    for path in ("src/gpu/" + f, "src/data/" + f, "include/dmlc/" + f):
        try:
            text = open(path).read().splitlines()[int(ln) - 1].strip()[:70]
            break
        except (OSError, IndexError, ValueError):
            pass
    print(f"{n:5d} {dict(kinds[line])!s:28s} {line:24s} {text}")
