"""Static check of counted waits in a gfx950 assembly listing (hipcc --cuda-device-only -S).

The fused MLP kernel (csrc/mlp_fused.hip) and the split-precision GEMMs (csrc/linear_x3.hip) issue
loads by inline asm and wait for them with hand-counted `s_waitcnt`: the compiler knows nothing about
the in-flight registers and may copy, spill or overwrite them at a merge before the wait.  Along every
control-flow path from each load, this checks:

* vm-reg   — a vector-memory load into VGPRs/AGPRs (buffer_/global_/flat_/scratch_load, returning
             atomics): no instruction reads or writes a destination register before an
             `s_waitcnt vmcnt(k)` with k <= the vector-memory ops (loads, stores, LDS-DMA) issued
             after the load on that path (they complete in order);
* lgkm-reg — an LDS read into VGPRs (ds_read*, ds_bpermute / ds_permute / ds_swizzle, ds_*_rtn):
             the same before an `s_waitcnt lgkmcnt(k)` with k <= the LDS ops issued after it (LDS ops
             complete in order among themselves; scalar-memory loads issued after it can complete
             first, so they never count as cover);
* dma      — an LDS-DMA load (`buffer_load_* ... lds`, `global_load_lds_*`): covered by a vmcnt wait
             before any s_barrier whose own block waited on vmcnt (the kernels' consumer barriers:
             "this chunk's weights have landed, then everyone's"); barriers without a vmcnt wait
             (e.g. the compositing hand-over) are passed through.

    hipcc -O3 -std=c++17 --offload-arch=gfx950 -I include -I csrc --cuda-device-only -S x.hip -o x.s
    python tools/check_inflight.py x.s [--all]

Loads emitted from inline asm (between ;;#ASMSTART / ;;#ASMEND) are flagged "asm".  Prints every
(load, first offending use) pair; exit status 1 if any.  tests/test_isa_waits.py runs it on every
translation unit that issues asm loads or waits.
"""
import re
import sys

VMEM = re.compile(r"^(buffer_|global_|flat_|scratch_)")
VM_LOAD = re.compile(r"^(?:buffer|global|flat|scratch)_(?:load|atomic)\w*\s+([va](?:\[\d+:\d+\]|\d+))")
DS_RET = re.compile(r"^ds_(?:read\w*|bpermute_b32|permute_b32|swizzle_b32|\w+_rtn\w*|consume|append)\s+"
                    r"([va](?:\[\d+:\d+\]|\d+))")
LGKM = re.compile(r"^(ds_|s_load|s_buffer_load|s_store|s_buffer_store|s_atomic|s_sendmsg|s_memtime|"
                  r"s_memrealtime|s_dcache|s_scratch)")
DS = re.compile(r"^ds_")
BRANCH = re.compile(r"^s_cbranch_\w+\s+(\S+)")
REG = re.compile(r"(?<![\w.])([va])(?:\[(\d+):(\d+)\]|(\d+)\b)")


def regset(text):
    out = set()
    for m in REG.finditer(text):
        k = m.group(1)
        if m.group(2) is not None:
            out |= {(k, r) for r in range(int(m.group(2)), int(m.group(3)) + 1)}
        else:
            out.add((k, int(m.group(4))))
    return out


def parse(path):
    """(instructions, labels, asm flags, function name per instruction)."""
    ins, labels, asm, func = [], {}, [], []
    in_asm, fn = False, "?"
    for raw in open(path):
        if ";;#ASMSTART" in raw:
            in_asm = True
        if ";;#ASMEND" in raw:
            in_asm = False
        t = raw.split(";")[0].strip()
        if not t:
            continue
        m = re.match(r"^([\w.$]+):", t)
        if m:
            labels[m.group(1)] = len(ins)
            if not m.group(1).startswith("."):
                fn = m.group(1)
            continue
        if t.startswith("."):
            continue
        ins.append(t)
        asm.append(in_asm)
        func.append(fn)
    return ins, labels, asm, func


def succ(ins, labels, i):
    t = ins[i]
    op = t.split()[0]
    if op == "s_endpgm" or op.startswith("s_setpc") or op.startswith("s_trap"):
        return []
    if op == "s_branch":
        return [labels[t.split()[1]]]
    m = BRANCH.match(t)
    if m and m.group(1) in labels:
        return [labels[m.group(1)], i + 1]
    return [i + 1]


def waits(t):
    """(vmcnt, lgkmcnt) of an s_waitcnt (None: that counter is not waited on)."""
    if not t.startswith("s_waitcnt"):
        return None, None
    vm = re.search(r"vmcnt\((\d+)\)", t)
    lg = re.search(r"lgkmcnt\((\d+)\)", t)
    if re.match(r"^s_waitcnt\s+0\s*$", t):
        return 0, 0
    return (int(vm.group(1)) if vm else None), (int(lg.group(1)) if lg else None)


def block_waited_vm(ins, labels_at, j):
    """Does the straight-line stretch before instruction j (back to a label or branch) wait on vmcnt?"""
    k = j - 1
    while k >= 0 and k not in labels_at:
        t = ins[k]
        if t.startswith("s_branch") or t.startswith("s_cbranch") or t.startswith("s_endpgm"):
            return False
        if waits(t)[0] is not None:
            return True
        k -= 1
    return False


SPAIR = re.compile(r"s\[(\d+):(\d+)\]")
SREG = re.compile(r"(?<![\w\[:])s(\d+)\b")


def sregs(text):
    out = set()
    for m in SPAIR.finditer(text):
        out |= set(range(int(m.group(1)), int(m.group(2)) + 1))
    for m in SREG.finditer(text):
        out.add(int(m.group(1)))
    return out


def track(u, consts, vcc):
    """Lane-mask flags the structurizer keeps in SGPR pairs: `s_mov_b64 s[a:b], -1 | 0` then
    `s_and(n2)_b64 vcc, exec, s[a:b]` + `s_cbranch_vcc(n)z` (exec is never zero in a live block).
    Returns the updated (known pair constants, known vcc) — any other mention of a pair forgets it."""
    m = re.match(r"^s_mov_b64\s+(s\[\d+:\d+\]),\s*(-1|0)$", u)
    if m:
        return consts - {c for c in consts if c[0] == m.group(1)} | {(m.group(1), int(m.group(2)))}, None
    m = re.match(r"^s_(and|andn2)_b64\s+vcc,\s*exec,\s*(s\[\d+:\d+\])$", u)
    if m:
        val = dict(consts).get(m.group(2))
        if val is None:
            return consts, None
        on = (val != 0) if m.group(1) == "and" else (val == 0)
        return consts, on
    if u.startswith(("s_nop", "s_waitcnt")):
        return consts, vcc
    used = sregs(u)
    if used:
        consts = frozenset(c for c in consts if not sregs(c[0]) & used)
    return consts, None


def succ_known(ins, labels, j, vcc):
    u = ins[j]
    if vcc is not None and u.startswith(("s_cbranch_vccnz", "s_cbranch_vccz")):
        take = vcc if u.startswith("s_cbranch_vccnz") else not vcc
        return [labels[u.split()[1]]] if take else [j + 1]
    return succ(ins, labels, j)


def walk(ins, labels, labels_at, i, kind, dst, cap, safe=None):
    """First offending instruction index on some path from load i, or None.  cap: one more than the
    largest count any wait of the listing names (counts past it are all covered alike).  safe: states
    already shown hazard-free (LDS-DMA walks do not depend on the load), shared across walks."""
    seen = set()
    dst = frozenset(dst)
    stack = [(j, 0, frozenset(), None, dst) for j in succ(ins, labels, i)]
    while stack:
        j, n, consts, vcc, live = stack.pop()
        if j >= len(ins) or (j, n, consts, vcc, live) in seen or (safe is not None and (j, n, consts, vcc) in safe):
            continue
        seen.add((j, n, consts, vcc, live))
        u = ins[j]
        vm, lg = waits(u)
        if kind in ("vm", "dma") and vm is not None and vm <= n:
            continue
        if kind == "lgkm" and lg is not None and lg <= n:
            continue
        if kind == "dma":
            if u.startswith("s_barrier") and block_waited_vm(ins, labels_at, j):
                return j
        else:
            touched = regset(u) & live
            if touched:
                # a later load of the same counter that only writes in-flight registers (reads none):
                # the returns land in issue order, so those registers end with the later value and
                # the earlier one is dead there; the rest stay in flight
                m = (VM_LOAD if kind == "vm" else DS_RET).match(u)
                if not m or regset(u[m.end():]) & live or not touched <= regset(m.group(1)):
                    return j
                live = live - touched
                if not live:
                    continue
        if kind == "lgkm":
            n2 = min(n + 1, cap) if DS.match(u) else n
        else:
            n2 = min(n + 1, cap) if VMEM.match(u) else n
        consts2, vcc2 = track(u, consts, vcc)
        for k in succ_known(ins, labels, j, vcc):
            stack.append((k, n2, consts2, vcc2, live))
    if safe is not None:
        safe.update((j, n, c, v) for j, n, c, v, _ in seen)
    return None


def functions(path):
    """Kernel (function) labels of a listing, in order."""
    return list(dict.fromkeys(parse(path)[3]))


def check(path, show_all=False, funcs=None):
    """(hazards, load counts) of the listing; funcs: only the loads of these functions."""
    ins, labels, asm, func = parse(path)
    labels_at = set(labels.values())
    caps = {"vm": 0, "lgkm": 0}
    for t in ins:
        vm, lg = waits(t)
        caps["vm"] = max(caps["vm"], vm or 0)
        caps["lgkm"] = max(caps["lgkm"], lg or 0)
    hits = []
    dma_safe = set()
    counts = {"vm": 0, "lgkm": 0, "dma": 0}
    for i, t in enumerate(ins):
        kind = dst = None
        if VMEM.match(t) and (" lds" in t or t.startswith("global_load_lds")):
            kind = "dma"
        else:
            m = VM_LOAD.match(t)
            if m and not (t.startswith(("buffer_atomic", "global_atomic", "flat_atomic")) and
                          not re.search(r"\b(sc0|glc)\b", t)):
                kind, dst = "vm", regset(m.group(1))
            else:
                m = DS_RET.match(t)
                if m:
                    kind, dst = "lgkm", regset(m.group(1))
        if kind is None or (funcs is not None and func[i] not in funcs):
            continue
        counts[kind] += 1
        j = walk(ins, labels, labels_at, i, kind, dst or set(), caps["lgkm" if kind == "lgkm" else "vm"] + 1,
                 dma_safe if kind == "dma" else None)
        if j is not None:
            hits.append((func[i], kind, asm[i], t, ins[j]))
    for fn, kind, is_asm, t, u in hits:
        print(f"[{kind}{' asm' if is_asm else ''}] {fn}\n   {t}\n   reached before its wait: {u}")
    if show_all or hits:
        print(f"{path}: checked {counts['vm']} vm loads, {counts['lgkm']} LDS reads, {counts['dma']} LDS-DMA loads; "
              f"{len(hits)} hazards")
    return hits, counts


def main(argv):
    paths = [a for a in argv if not a.startswith("--")]
    bad = 0
    for p in paths:
        hits, counts = check(p, show_all="--all" in argv)
        bad += len(hits)
        if not hits and "--all" not in argv:
            print(f"{p}: {counts['vm']} vm loads, {counts['lgkm']} LDS reads, {counts['dma']} LDS-DMA loads: ok")
    return 1 if bad else 0


if __name__ == "__main__":
    sys.exit(main(sys.argv[1:]))
