"""Static instruction mix of one kernel in a hipcc -S listing.
usage: python scripts/asm_stats.py file.s <substring of kernel symbol>"""
import collections
import re
import sys

s = open(sys.argv[1]).read().splitlines()
key = sys.argv[2]
start = next(i for i, l in enumerate(s) if re.match(r"^_Z\S*" + re.escape(key) + r"\S*:", l))
end = next(i for i in range(start, len(s)) if s[i].startswith(".Lfunc_end"))
ins = [l.strip() for l in s[start:end] if l.startswith("\t") and not l.strip().startswith((".", ";"))]
c = collections.Counter(x.split()[0] for x in ins)
print(s[start][:120])
print("static instructions", len(ins))
print("VALU", sum(v for k, v in c.items() if k.startswith("v_")),
      "SALU", sum(v for k, v in c.items()
                  if k.startswith("s_") and not k.startswith(("s_waitcnt", "s_cbranch", "s_branch"))),
      "DS", sum(v for k, v in c.items() if k.startswith("ds_")),
      "VMEM", sum(v for k, v in c.items() if k.startswith(("global_", "buffer_", "flat_"))),
      "branches", sum(v for k, v in c.items() if "branch" in k))
print(c.most_common(int(sys.argv[3]) if len(sys.argv) > 3 else 40))
