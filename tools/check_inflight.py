"""Check a gfx950 assembly listing for uses of a buffer load's destination VGPRs before a
`s_waitcnt vmcnt` that covers the load, along every control-flow path (the fused MLP kernel
issues loads by inline asm with hand-counted waits: the compiler knows nothing about the
in-flight registers and may copy or overwrite them at a merge).

    hipcc -O3 --offload-arch=gfx950 --cuda-device-only -S csrc/mlp_fused.hip -o /tmp/mf.s
    python tools/check_inflight.py /tmp/mf.s

A load is covered by `s_waitcnt vmcnt(N)` once at least N vector-memory operations were issued
after it on that path (they complete in order).  Prints every (load, use) pair found; exit 1 if any.
"""
import re
import sys

VMEM = re.compile(r"^(buffer_|global_|flat_|scratch_)")
LOAD = re.compile(r"^(?:buffer|global)_load_dword(?:x\d)?\s+v\[(\d+):(\d+)\]")


def regs(text):
    out = set()
    for m in re.finditer(r"v\[(\d+):(\d+)\]", text):
        out |= set(range(int(m.group(1)), int(m.group(2)) + 1))
    for m in re.finditer(r"(?<![\w\[:])v(\d+)\b", text):
        out.add(int(m.group(1)))
    return out


def parse(path):
    ins, labels = [], {}
    for raw in open(path):
        t = raw.split(";")[0].strip()
        if not t or t.startswith("."):
            m = re.match(r"^(\.L\w+):", t)
            if m:
                labels[m.group(1)] = len(ins)
            continue
        m = re.match(r"^([\w.$]+):$", t)
        if m:
            labels[m.group(1)] = len(ins)
            continue
        ins.append(t)
    return ins, labels


def succ(ins, labels, i):
    t = ins[i]
    op = t.split()[0]
    if op == "s_endpgm" or op.startswith("s_setpc") or op.startswith("s_trap"):
        return []
    if op == "s_branch":
        return [labels[t.split()[1]]]
    if op.startswith("s_cbranch"):
        return [labels[t.split()[1]], i + 1]
    return [i + 1]


def main(path):
    ins, labels = parse(path)
    bad = 0
    for i, t in enumerate(ins):
        m = LOAD.match(t)
        if not m or " lds" in t:
            continue
        dst = set(range(int(m.group(1)), int(m.group(2)) + 1))
        seen = set()
        stack = [(j, 0) for j in succ(ins, labels, i)]
        hits = []
        while stack:
            j, n = stack.pop()
            if j >= len(ins) or (j, n) in seen:
                continue
            seen.add((j, n))
            u = ins[j]
            w = re.search(r"vmcnt\((\d+)\)", u) if u.startswith("s_waitcnt") else None
            if w and int(w.group(1)) <= n:
                continue
            if regs(u) & dst:
                hits.append(u)
                continue
            n2 = min(n + 1, 64) if VMEM.match(u) else n
            for k in succ(ins, labels, j):
                stack.append((k, n2))
        if hits:
            bad += 1
            print(f"load #{i}: {t}\n   used before its wait: {sorted(set(hits))[:4]}")
    print(f"{bad} loads with uses before their wait")
    return 1 if bad else 0


if __name__ == "__main__":
    sys.exit(main(sys.argv[1]))
