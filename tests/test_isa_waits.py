"""Counted-wait discipline of the inline-asm loads, checked on the compiled gfx950 ISA (CPU: hipcc
cross-compiles, nothing runs).  The fused field-MLP kernel (csrc/mlp_fused.hip: the forward and the
input-gradient chain of barf/model_interpolation_architecture.py:96-141), the split-precision GEMMs
(csrc/linear_x3.hip) and the resample (csrc/sampling.hip) issue buffer loads, LDS reads and LDS-DMA by
inline asm and wait for them with hand-counted `s_waitcnt`; hipcc does not know those registers are in
flight and may copy or reuse them before the wait.  tools/check_inflight.py walks every control-flow
path from every load (asm or compiler-issued) in the ISA of each translation unit and fails on:
* a destination VGPR touched before a covering `vmcnt` (vector-memory loads) or `lgkmcnt` (LDS reads);
* an LDS-DMA not covered by a vmcnt wait at the next consumer barrier.
The checker itself is pinned on small synthetic listings (hazard found / covered / infeasible path)."""
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "nerf-experiments_amd")
sys.path.insert(0, os.path.join(ROOT, "tools"))
import check_inflight as C  # noqa: E402

HIPCC = "/opt/rocm/bin/hipcc"
TUS = ["mlp_fused", "linear_x3", "sampling"]


def _listing(tmp_path, text):
    p = tmp_path / "t.s"
    p.write_text(text)
    return str(p)


def test_checker_flags_use_before_vmcnt(tmp_path):
    s = _listing(tmp_path, """k:
  ;;#ASMSTART
  buffer_load_dwordx4 v[4:7], v1, s[0:3], 0 offen
  ;;#ASMEND
  buffer_store_dword v2, v1, s[0:3], 0 offen
  s_waitcnt vmcnt(1)
  v_mov_b32_e32 v8, v5
  s_endpgm
""")
    hits, _ = C.check(s)
    assert len(hits) == 0           # one younger store: vmcnt(1) covers the load
    s = _listing(tmp_path, """k:
  buffer_load_dwordx4 v[4:7], v1, s[0:3], 0 offen
  s_waitcnt vmcnt(1)
  v_mov_b32_e32 v8, v5
  s_endpgm
""")
    hits, _ = C.check(s)
    assert len(hits) == 1 and hits[0][1] == "vm"


def test_checker_flags_lds_read_before_lgkmcnt_and_ignores_smem_cover(tmp_path):
    s = _listing(tmp_path, """k:
  ds_read_b128 v[4:7], v1
  s_load_dword s4, s[0:1], 0x0
  s_waitcnt lgkmcnt(1)
  v_mfma_f32_16x16x32_bf16 v[8:11], v[4:7], v[12:15], 0
  s_endpgm
""")
    hits, _ = C.check(s)
    assert len(hits) == 1 and hits[0][1] == "lgkm"     # the scalar load may complete first
    s = _listing(tmp_path, """k:
  ds_read_b128 v[4:7], v1
  ds_read_b128 v[16:19], v1 offset:1024
  s_waitcnt lgkmcnt(1)
  v_mfma_f32_16x16x32_bf16 v[8:11], v[4:7], v[12:15], 0
  s_endpgm
""")
    assert len(C.check(s)[0]) == 0


def test_checker_flags_dma_before_consumer_barrier(tmp_path):
    base = """k:
  buffer_load_dwordx4 v148, s[28:31], s16 offen lds
  buffer_store_dwordx4 v[0:3], v1, s[0:3], 0 offen
  s_waitcnt lgkmcnt(0)
  s_barrier
  s_waitcnt vmcnt(%d)
  s_waitcnt lgkmcnt(0)
  s_barrier
  ds_read_b128 v[4:7], v2
  s_endpgm
"""
    # the first barrier has no vmcnt wait (a hand-over barrier): passed through
    assert len(C.check(_listing(tmp_path, base % 1))[0]) == 0
    hits, _ = C.check(_listing(tmp_path, base % 2))
    assert len(hits) == 1 and hits[0][1] == "dma"


def test_checker_resolves_structurizer_flags(tmp_path):
    # the two store blocks are exclusive: s[14:15] = -1 only when the first is skipped
    s = _listing(tmp_path, """k:
  buffer_load_dwordx4 v148, s[28:31], s16 offen lds
  s_mov_b64 s[14:15], -1
  s_cmp_lt_i32 s90, 0
  s_cbranch_scc1 .LB1
  buffer_store_dwordx4 v[0:3], v1, s[0:3], 0 offen
  s_mov_b64 s[14:15], 0
.LB1:
  s_andn2_b64 vcc, exec, s[14:15]
  s_cbranch_vccnz .LB2
  buffer_store_dwordx4 v[0:3], v1, s[0:3], 0 offen
.LB2:
  s_waitcnt vmcnt(1)
  s_barrier
  s_endpgm
""")
    assert len(C.check(s)[0]) == 0


def _compile(tu, out_dir):
    out = os.path.join(out_dir, f"{tu}.s")
    cmd = [HIPCC, "-O3", "-std=c++17", "--offload-arch=gfx950", "-I", os.path.join(ROOT, "include"), "-I",
           os.path.join(PKG, "csrc"), "--cuda-device-only", "-S", os.path.join(PKG, "csrc", f"{tu}.hip"), "-o", out]
    subprocess.run(cmd, check=True, capture_output=True, timeout=600)
    return out


@pytest.fixture(scope="module")
def listings(tmp_path_factory):
    if not os.path.exists(HIPCC):
        pytest.skip("hipcc not installed")
    d = str(tmp_path_factory.mktemp("isa"))
    return {tu: _compile(tu, d) for tu in TUS}


def _check_fn(args):
    path, fn = args
    return C.check(path, funcs={fn})


@pytest.mark.parametrize("tu", TUS)
def test_product_isa_has_no_wait_hazard(tu, listings):
    from concurrent.futures import ProcessPoolExecutor
    fns = C.functions(listings[tu])
    with ProcessPoolExecutor(max_workers=min(8, os.cpu_count() or 1)) as ex:
        res = list(ex.map(_check_fn, [(listings[tu], fn) for fn in fns]))
    hits = [h for r in res for h in r[0]]
    counts = {k: sum(r[1][k] for r in res) for k in ("vm", "lgkm", "dma")}
    assert sum(counts.values()) > 0
    assert not hits, "\n".join(f"[{k}] {fn}: {t} -> {u}" for fn, k, _, t, u in hits[:10])
    if tu == "mlp_fused":
        assert counts["dma"] > 0 and counts["lgkm"] > 0 and counts["vm"] > 0


def test_checker_catches_weakened_asm_waits(listings, tmp_path):
    """Mutation: the fused kernel's listing with every inline-asm wait count raised by 6 (one chunk's
    worth of loads and stores too few) must fail on all three counts: the check is not vacuous on the
    real code."""
    import re
    keep, in_asm = [], False
    for ln in open(listings["mlp_fused"]).read().split("\n"):
        if ";;#ASMSTART" in ln:
            in_asm = True
        if ";;#ASMEND" in ln:
            in_asm = False
        if in_asm and ln.strip().startswith("s_waitcnt"):
            ln = re.sub(r"(vmcnt|lgkmcnt)\((\d+)\)", lambda m: f"{m.group(1)}({min(int(m.group(2)) + 6, 15)})", ln)
        keep.append(ln)
    p = tmp_path / "mutant.s"
    p.write_text("\n".join(keep))
    hits, _ = C.check(str(p))
    kinds = {k for _, k, _, _, _ in hits}
    assert {"vm", "lgkm", "dma"} <= kinds, kinds
