"""Instruction histogram of one loop body of a kernel in a hipcc -S output.

    python tools/asmhist.py file.s <kernel-substring> <loop label>
"""
import collections
import re
import sys

s = open(sys.argv[1]).read()
f = [x for x in re.split(r"\n(?=_Z\w+:)", s) if sys.argv[2] in x.split(":", 1)[0]][0]
lines = f.split("\n")
lab = sys.argv[3]
start = [i for i, l in enumerate(lines) if l.startswith(lab + ":")][0]
end = [i for i, l in enumerate(lines) if i > start and re.search(r"s_cbranch\w*\s+" + lab + r"\b", l)][0]
body = [l.strip() for l in lines[start:end + 1] if l.strip() and not l.strip().startswith((";", "."))]
for k, v in collections.Counter(l.split()[0] for l in body).most_common():
    print(v, k)
print(len(body), "instructions")
