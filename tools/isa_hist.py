"""Instruction histogram of the main loop of a kernel in a --save-temps .s file.
usage: isa_hist.py FILE.s SYMBOL_SUBSTRING [top]"""
import collections
import re
import sys

s = open(sys.argv[1]).read()
pat = sys.argv[2]
top = int(sys.argv[3]) if len(sys.argv) > 3 else 45
m = re.search(r"^(_Z\w*" + re.escape(pat) + r"\w*):.*?\n(.*?)\n\s*s_endpgm", s, re.S | re.M)
body = m.group(2).split("\n")
labels = {l.split(":")[0]: i for i, l in enumerate(body) if re.match(r"^\.LBB\w+:", l)}
loops = []
for i, l in enumerate(body):
    mm = re.match(r"\s*s_(?:cbranch_\w+|branch)\s+(\.LBB\w+)", l)
    if mm and mm.group(1) in labels and labels[mm.group(1)] < i:
        loops.append((labels[mm.group(1)], i))
a, b = max(loops, key=lambda t: t[1] - t[0])
c = collections.Counter()
for l in body[a:b + 1]:
    t = l.strip().split()
    if t and not t[0].startswith((".", ";")):
        c[t[0]] += 1
print(m.group(1), "loop lines", a, b)
print("VALU", sum(v for k, v in c.items() if k.startswith("v_")), "DS",
      sum(v for k, v in c.items() if k.startswith("ds_")), "SALU",
      sum(v for k, v in c.items() if k.startswith("s_")), "total", sum(c.values()))
for k, v in c.most_common(top):
    print(f"{k:28s}{v}")
