"""Instruction mix per basic block of one kernel in a hipcc -S listing (loop bodies are the
large blocks): python tools/isa_mix.py <file.s> <symbol substring>"""
import collections
import re
import sys

s = open(sys.argv[1]).read()
m = re.search(r"^(_Z\S*" + re.escape(sys.argv[2]) + r"\S*):", s, re.M)
start = m.start()
end = s.index(".Lfunc_end", start)
blocks, cur, name = [], [], "entry"
for line in s[start:end].split("\n"):
    if re.match(r"^\.LBB\d+_\d+:", line):
        blocks.append((name, cur))
        cur, name = [], line.split()[0]
    else:
        cur.append(line)
blocks.append((name, cur))
for name, b in blocks:
    ins = [l.strip().split()[0] for l in b if l.startswith("\t") and not l.strip().startswith((";", "."))]
    c = collections.Counter()
    for x in ins:
        k = ("mfma" if x.startswith("v_mfma") else "valu" if x.startswith("v_") else "salu" if x.startswith("s_")
             else "lds" if x.startswith("ds_") else "vmem" if x.startswith(("global_", "buffer_")) else "other")
        c[k] += 1
    if len(ins) > 20:
        print(name, len(ins), dict(c))
        if len(sys.argv) > 3:
            print(collections.Counter(x for x in ins if x.startswith("v_") and not x.startswith("v_mfma")).most_common(25))
