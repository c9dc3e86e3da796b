"""Per-block instruction classes of the loop blocks of one kernel in a hipcc -S listing:
python tools/isa_loop.py <file.s> <symbol substring> [--valu]"""
import collections
import re
import sys

s = open(sys.argv[1]).read()
m = re.search(r"^(_Z\S*" + re.escape(sys.argv[2]) + r"\S*):", s, re.M)
body = s[m.start():s.index(".Lfunc_end", m.start())].split("\n")
blocks, name, tag, cnt, vv = [], "entry", "", collections.Counter(), collections.Counter()
for line in body:
    mm = re.match(r"^(\.LBB\d+_\d+|; %bb\.\d+):(.*)", line)
    if mm:
        blocks.append((name, tag, cnt, vv))
        name, tag, cnt, vv = mm.group(1), mm.group(2).strip(), collections.Counter(), collections.Counter()
        continue
    t = line.strip().split()
    if not t or t[0].startswith((";", ".")):
        continue
    x = t[0]
    k = ("mfma" if x.startswith("v_mfma") else "valu" if x.startswith("v_") else "salu" if x.startswith("s_")
         else "lds" if x.startswith("ds_") else "vmem" if x.startswith(("global_", "buffer_")) else "other")
    cnt[k] += 1
    if k == "valu":
        vv[x] += 1
blocks.append((name, tag, cnt, vv))
for name, tag, c, v in blocks:
    if "Loop" in tag:
        print(name, tag.split("Header=")[-1][:20], dict(c))
        if "--valu" in sys.argv:
            print("    ", v.most_common(10))
