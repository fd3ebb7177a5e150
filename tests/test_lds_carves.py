"""LDS carves of every kernel family, checked on the host over size sweeps.

Each kernel carves its dynamic LDS into regions with a ``carve()`` shared by
host and device; ``dr_debug_carve_*`` (C ABI, host-only) reports the offsets.
For every family and sweep point:

* every region starts 16-byte aligned, inside the carve;
* regions are disjoint: a region's size is the distance to the next distinct
  offset (or the carve's end), and must cover the extent the kernel touches —
  restated below from the kernels' index arithmetic (file:line), independently
  of the TAKE sizes.  Two fields may share an offset only where the kernel
  aliases them on purpose (listed per family);
* the carve's total equals the bytes the host reserves for the launch
  (``dr_*_lds_bytes``), and the host's "fits 160 KiB" decision is the carve's.

A region written past its end (r03's a84ddda: a FoutNet head-backward region
sized for 16 chunks and written with 32) fails the extent check.
"""

from __future__ import annotations

import ctypes

import pytest

from deeprank2_amd import _lib

LDS_MAX = 160 * 1024


def r4(v):
    return (v + 3) & ~3


def r16(v):
    return (v + 15) & ~15


def _carve(kind, q):
    lib = _lib.load()
    arr = (ctypes.c_int32 * len(q))(*q)
    buf = ctypes.create_string_buffer(8192)
    n = getattr(lib, f"dr_debug_carve_{kind}")(arr, buf, 8192)
    assert 0 < n < 8192
    vals = {}
    for part in buf.value.decode().split(";"):
        if part:
            k, v = part.split("=")
            vals[k] = int(v)
    return vals


def _regions(vals, fields=None):
    total = vals["total"]
    offs = {k: v for k, v in vals.items() if k != "total" and not k.startswith("$") and (fields is None or k in fields)}
    ends = sorted(set(offs.values()) | {total})
    size = {}
    for k, o in offs.items():
        assert 0 <= o <= total, (k, o, total)
        assert o % 4 == 0, (k, o)
        size[k] = ends[ends.index(o) + 1] - o if o < total else 0
    return offs, size, total


def _check(kind, q, extents, aliases=(), host_bytes=None, phases=()):
    """phases: groups of fields that overlay the same LDS at different times
    (a kernel's forward and backward edge buffers, staging reused later);
    every group is checked with the fields outside all groups."""
    vals = _carve(kind, q)
    ext = extents(vals)
    in_phase = set().union(*phases) if phases else set()
    common = {k for k in vals if k != "total" and not k.startswith("$")} - in_phase
    total = vals["total"]
    for group in phases or [set()]:
        offs, size, total = _regions(vals, common | set(group))
        for k, need in ext.items():
            if k in offs:
                assert size[k] >= need, f"{kind}{tuple(q)}: region {k} has {size[k]} words, the kernel touches {need}"
        # shared offsets only between declared aliases or with empty regions
        by_off = {}
        for k, o in offs.items():
            by_off.setdefault(o, []).append(k)
        for o, names in by_off.items():
            live = [k for k in names if ext.get(k, 0) > 0]
            if len(live) > 1:
                assert any(set(live) <= set(a) for a in aliases), f"{kind}{tuple(q)}: {live} overlap at {o}"
    if host_bytes is not None:
        assert 4 * total == host_bytes, (kind, q, 4 * total, host_bytes)
    return vals, total


# ---- GINet per-graph kernel (ginet_fused.hip:67-109; graph_body :560-838) ----
def _ginet_ext(N, E, F, K0, P1, K1, alias, OUT):
    def ext(v):
        KP = 32 if F <= 32 else 64  # the kernel's KPT: rows as wide as its MFMA steps (r05)
        XS, LDW = r4(F), KP + 2
        assert (v["$XS"], v["$KP"], v["$LDW"]) == (XS, KP, LDW)
        e = {
            "w1": 32 * F,  # dma_words(sW1, w1, 16F) + (sW1 + 16F, w1e, 16F) (:632-633)
            "w2": 1024,  # sW2[tid], tid < NT (:766)
            "fc2": OUT * 128 + OUT,  # sFc2[tid + u NT] < nf (:768-771)
            "x": N * XS,  # dma_x4(sX, .., N XS / 4) (:620)
            "z": N * LDW,  # rows i < N, columns < KPT (:634-639, :704-716)
            "rp": N + 1,
            "col": ((E + 7) // 8) * 4,  # dma_x4 of (E + 7) / 8 16-byte units of uint16 ids (:621)
            "cl0": N,
            "key": 2 * K0 * 32,  # 64-bit keys [K0][32] (:640, :747)
            "p1": K0 * 32,
            "a1": K0 * 32,  # sP1 / sA1[p], p < K0 * 32 (:824-828)
            "dp1": K0 * 32,
            "y2": K0 * 64,
            "h2": K0 * 64,
            "p1rp": K0 + 1,
            "p1c": P1,
            "m1p": K1 + 1,
            "m1i": K0,
            "p2": K1 * 64,
            "nt": K1 * 64,
            "cl1": K0,
            "head": 672,  # HEADW: G64 hpre128 hh128 hd128 dh128 dG64 dout16 spare16
            "dgp": 16 * 64,  # [NW][64] head-backward partials
            "keep": 32,  # 128 keep bytes (:762-765)
        }
        if not alias:
            e |= {"p1trp": K0 + 1, "p1tc": P1}
        return e

    return ext


@pytest.mark.parametrize(("N", "E", "K0", "P1", "K1", "alias", "OUT"), [(1, 0, 1, 0, 1, 1, 1), (30, 120, 3, 6, 1, 1, 2), (200, 3000, 5, 14, 1, 1, 1), (220, 4400, 6, 22, 2, 0, 16), (170, 11900, 1, 0, 1, 1, 2)])
@pytest.mark.parametrize("F", [1, 30, 50])
def test_ginet_graph_carve(N, E, F, K0, P1, K1, alias, OUT):
    q = [N, E, F, K0, P1, K1, alias, OUT]
    _check("ginet", q, _ginet_ext(*q), aliases=[("p1rp", "p1trp"), ("p1c", "p1tc")], host_bytes=_lib.load().dr_ginet_lds_bytes(*q))


# ---- GINet large-graph tile / tail kernels (ginet_fused.hip:990-1030, :1292-1330, :1479-1525) ----
TR = 128  # DR_LARGE_TILE


@pytest.mark.parametrize(("N", "F", "K0", "HM", "EM"), [(3000, 30, 32, 0, 0), (3000, 30, 32, 600, 2400), (900, 50, 8, 300, 1200), (16, 1, 1, 16, 30)])
def test_ginet_large_conv_carves(N, F, K0, HM, EM):
    def ext(v):
        XS, LDW = r4(F), r16(F) + 2
        # flg: one word per tile row, the pooling-arg flags of conv_tile_f32 (r06)
        e = {"w1": 32 * LDW, "z": TR * LDW, "m0i": TR if HM else N, "m0p": K0 + 1, "rng": 2 * K0, "flg": TR, "hid": HM}
        if HM:
            e |= {"xh": max(HM * XS, TR * 32), "trp": TR + 1, "lcol": (EM + 8) // 2}
        else:
            e["h"] = TR * 32
        return e

    q = [N, F, K0, HM, EM]
    _check("ginet_conv", q, ext, aliases=[("h", "xh")], host_bytes=_lib.load().dr_ginet_large_conv_lds_bytes(*q))

    def ext_b(v):
        KPB = (F + 31) & ~31
        ZSB, XSB = KPB + 8, (F + 7) & ~7
        e = {"w1": 32 * ZSB // 2, "z": TR * ZSB // 2, "h": TR * 32, "m0i": TR if HM else N, "m0p": K0 + 1, "rng": 2 * K0, "flg": TR, "hid": HM}
        if HM:
            e |= {"xh": HM * XSB // 2, "trp": TR + 1, "lcol": (EM + 8) // 2}
        return e

    _check("ginet_conv_bf16", q, ext_b, host_bytes=_lib.load().dr_ginet_large_conv_lds_bytes_bf16(*q))


@pytest.mark.parametrize(("K0", "P1", "K1", "alias", "OUT"), [(1, 0, 1, 1, 1), (32, 200, 1, 1, 2), (32, 200, 3, 0, 16)])
def test_ginet_tail_carve(K0, P1, K1, alias, OUT):
    def ext(v):
        e = {"w2": 1024, "fc2": OUT * 128 + OUT, "p1": K0 * 32, "a1": K0 * 32, "dp1": K0 * 32, "y2": K0 * 64, "h2": K0 * 64, "p1rp": K0 + 1, "p1c": P1, "m1p": K1 + 1, "m1i": K0, "p2": K1 * 64, "nt": K1 * 64, "cl1": K0, "head": 672, "dgp": 16 * 64}
        if not alias:
            e |= {"p1trp": K0 + 1, "p1tc": P1}
        return e

    q = [K0, P1, K1, alias, OUT]
    _check("ginet_tail", q, ext, aliases=[("p1rp", "p1trp"), ("p1c", "p1tc")], host_bytes=_lib.load().dr_ginet_tail_lds_bytes(*q))


# ---- FoutNet / SGAT per-graph kernel (fout_fused.hip:44-128; body :420-650) ----
@pytest.mark.parametrize(("N", "E", "K0", "P1", "K1", "alias", "OUT"), [(1, 0, 1, 0, 1, 1, 1), (200, 3000, 5, 14, 1, 1, 1), (268, 4000, 6, 22, 2, 0, 4), (171, 11900, 1, 0, 1, 1, 2)])
@pytest.mark.parametrize(("F", "sg"), [(30, 0), (50, 0), (30, 1)])
def test_fout_graph_carve(N, E, F, K0, P1, K1, alias, OUT, sg):
    q = [N, E, F, K0, P1, K1, alias, OUT]
    host = (_lib.load().dr_sgat_lds_bytes if sg else _lib.load().dr_fout_lds_bytes)(*q)

    def ext(v):
        XS, KP = r4(F), r16(2 * F)
        wide = bool(v["$wide"])
        LDZ = 2 * XS + 2 if wide else XS + 2
        assert v["$LDZ"] == LDZ
        e = {
            "wc1": KP * 16,
            "w2": 16 * 32 * 2 + 32 + 16,
            "fc1": 64 * 32 + 64,
            "fc2": OUT * 64 + OUT,
            "x": N * XS,
            "zm": N * LDZ,
            "h1": N * 16,
            "rp": N + 1,
            "col": ((E + 7) // 8) * 4,  # dma_x4 of (E + 7) / 8 16-byte units (:477)
            "m0p": K0 + 1,
            "m0i": N,
            "p1": K0 * 16,
            "a1": K0 * 16,
            "dp1": K0 * 16,
            "zm2": K0 * 16,
            "s2": K0 * 32,
            "h2": K0 * 32,
            "d2": K0 * 32,
            "dz2": K0 * 16,
            "p1rp": K0 + 1,
            "p1c": P1,
            "m1p": K1 + 1,
            "m1i": K0,
            "p2": K1 * 32,
            "nt": K1 * 32,
            "head": 512,  # HEADW
            "dgp": 1024,  # the head backward's [NT / 32 chunks][32] partials (the a84ddda region)
            "red": 2 * 1024,  # tb = sRed, ta = sRed + NT (:598-599)
        }
        if not alias:
            e |= {"p1trp": K0 + 1, "p1tc": P1}
        if sg:
            e |= {"ea": E, "c1": N, "p1w": P1, "p1tid": P1, "c2": K0}
        return e

    vals, total = _check("fout", [*q, sg, LDS_MAX], ext, aliases=[("p1rp", "p1trp"), ("p1c", "p1tc")], host_bytes=host)
    # the wide [x | Zm] layout exactly when it fits 160 KiB (carve(), fout_fused.hip:122-128)
    if not vals["$wide"]:
        wide_words = _carve("fout", [*q, sg, 1 << 30])["total"]
        assert 4 * wide_words > LDS_MAX


@pytest.mark.parametrize(("N", "F", "K0", "HM", "EM", "sg"), [(3000, 30, 32, 600, 2400, 0), (3000, 30, 32, 600, 2400, 1), (2800, 50, 16, 0, 0, 0)])
def test_fout_large_carves(N, F, K0, HM, EM, sg):
    TRF = TR

    def ext(v):
        KP = r16(2 * F)
        e = {"w": KP * 16, "b1": 16, "a": TRF * (KP + 4), "h": TRF * 16, "c1": TRF if sg else 0, "m0i": TRF if HM else N, "m0p": K0 + 1, "flg": TRF, "xh": HM * r4(F), "hid": HM, "trp": TRF + 1 if HM else 0, "lcol": (EM + 8) // 2 if HM else 0}
        return e

    q = [N, F, K0, HM, EM, sg]
    _check("fout_conv", q, ext, host_bytes=_lib.load().dr_fout_large_conv_lds_bytes(*q))

    def ext_t(v, K0=K0):
        P1, K1, OUT = 3 * K0, 2, 2
        e = {"w2": 16 * 32 * 2 + 32 + 16, "fc1": 64 * 32 + 64, "fc2": OUT * 64 + OUT, "p1": K0 * 16, "a1": K0 * 16, "dp1": K0 * 16, "zm2": K0 * 16, "s2": K0 * 32, "h2": K0 * 32, "d2": K0 * 32, "dz2": K0 * 16, "p1rp": K0 + 1, "p1c": P1, "p1trp": K0 + 1, "p1tc": P1, "m1p": K1 + 1, "m1i": K0, "p2": K1 * 32, "nt": K1 * 32, "head": 512, "dgp": 16 * 64}
        if sg:
            e |= {"p1w": P1, "p1tid": P1, "c2": K0}
        return e

    qt = [K0, 3 * K0, 2, 0, 2, sg]
    _check("fout_tail", qt, ext_t, host_bytes=_lib.load().dr_fout_tail_lds_bytes(*qt))


# ---- ginet_nocluster per-graph kernel (ginet_nocluster.hip:39-110) ----
@pytest.mark.parametrize(("N", "E", "F", "OUT"), [(1, 0, 30, 1), (200, 3000, 30, 1), (220, 4400, 50, 16)])
def test_nocluster_carve(N, E, F, OUT):
    def ext(v):
        return {"rp": N + 1, "trp": N + 1, "col": (E + 1) // 2, "tcol": (E + 1) // 2, "head": 672}

    q = [N, E, F, OUT]
    _check("nocluster", q, ext, host_bytes=_lib.load().dr_ginet_nocluster_lds_bytes(*q))


# ---- VanillaNetwork per-graph kernel (vanilla_graph.hip:66-100) ----
@pytest.mark.parametrize(("N", "E"), [(1, 0), (3, 3), (200, 3000), (220, 4400)])
@pytest.mark.parametrize("Fe", [0, 1, 3, 4])
def test_vanilla_graph_carve(N, E, Fe):
    LS = 34

    def ext(v):
        # P and T hold node rows (stride LS) or the D pass partials + its edge buffer
        slot = max(r4(N * LS), 16 * 32 * (1 + Fe) + 1024, 1024)
        # forward: 16-byte edge records + 16 zero records (a row pass reads up to
        # 15 past its row), the 4th edge feature behind them; backward: T, the
        # ReLU words, the transposed CSR
        return {"rp": N + 1, "xb": N, "head": 512, "P": slot, "Q": N * LS, "R": N * LS, "U": 4 * (E + 16), "ext": (E + 16) if Fe > 3 else 0, "T": slot, "bt": E, "trp": N + 1, "tcol": (E + 1) // 2}

    q = [N, E, Fe]
    _check("vanilla_graph", q, ext, host_bytes=_lib.load().dr_vanilla_fused_lds_bytes(*q), phases=[{"U", "ext"}, {"T", "bt", "trp", "tcol"}])


# ---- Vanilla pipeline: 16/32-row edge tiles and the chunk-fused kernels (vanilla_fused.hip) ----
@pytest.mark.parametrize(("H", "EM", "TM"), [(1, 1, 1), (72, 559, 559), (155, 1855, 1855), (400, 6000, 6000)])
@pytest.mark.parametrize("Fe", [0, 1, 3, 4])
def test_vanilla_tile_and_chunk_carves(H, EM, TM, Fe):
    RS = 4 if Fe <= 3 else 8
    for bwd in (0, 1):
        _check("vanilla_tile", [H, EM, TM, Fe, bwd], lambda v, bwd=bwd: {"rec": EM * RS} | ({"trec": 2 * TM} if bwd else {}))
    F = 30
    XS = r4(F)
    # vc_fwd (both layers): own X rows (-> A in place) and halo X rows (-> B in place) at
    # stride 36 (halo rounded up to 16-row MFMA blocks), [Wa; Wb]^T [XS][64], CSR records;
    # after the edge phase the same space holds [X | S] rows at KP + 4, Wn^T [KP][NOP], bn
    def fext(v):
        KP = XS + 32
        return {"xo": 64 * 36, "wab": XS * 64, "halo": r16(H) * 36, "rec": EM * RS, "a": 64 * (KP + 4), "wn": KP * r16(F), "bn": r16(F), "x2": 64 * 33}

    vals, total = _check("vanilla_chunk_fwd", [F, H, EM, Fe], fext, phases=[{"xo", "wab", "halo", "rec"}, {"a", "wn", "bn", "x2"}])
    assert vals["a"] == 0 and vals["x2"] + 64 * 33 <= total
    FeS = max(Fe, 1)
    for two in (0, 1):
        # vc_eb2n1 / vc_eb1: [D | D'] rows (LDD 68), (vc_eb2n1) [Wa2; Wb2] [64][NOP3] and DU1 at
        # XS + 4, the waves' dWc shares sSh[(wave 32 + c) FeS + f], halo dS rows and transposed
        # {col, word} records (the CSR records stay in registers); after the edge phase the same
        # space holds X0 rows and (vc_eb2n1) X1 / dX1 / S1 rows and Wn1[:, F:]^T [XS][32]
        def bext(v, two=two):
            e = {"d": 64 * 68, "sh": 16 * 32 * FeS, "halo": H * 32, "trec": 2 * TM, "x0": 64 * XS}
            if two:
                e |= {"w3": 64 * r16(F), "du": 64 * (XS + 4), "x1": 64 * XS, "dx": 64 * XS, "s1": 64 * 32, "w1": XS * 32}
            return e

        late = {"x0", "x1", "dx", "s1", "w1"}  # (vc_eb1: x1 .. w1 empty)
        vals, total = _check("vanilla_chunk_bwd", [F, H, EM, TM, Fe, two], bext, phases=[{"halo", "trec"}, late])
        assert vals["x0"] == vals["halo"]  # the late rows overlay the dead edge space
        if two:
            assert vals["w1"] + XS * 32 <= total


# ---- tile order of the tile kernels (graph_common.h xcd_tile_of, r06) ----
@pytest.mark.parametrize("n", [1, 7, 8, 9, 64, 255, 642, 1528, 3001])
def test_xcd_tile_order_is_a_contiguous_permutation(n):
    lib = _lib.load()
    out = (ctypes.c_int32 * n)()
    assert lib.dr_debug_xcd_tile(n, out) == 0
    tiles = list(out)
    assert sorted(tiles) == list(range(n))  # every tile run exactly once
    for x in range(8):  # blocks b, b + 8, ... (one XCD under round-robin dispatch) take consecutive tiles
        mine = tiles[x::8]
        assert mine == list(range(mine[0], mine[0] + len(mine))) if mine else True
