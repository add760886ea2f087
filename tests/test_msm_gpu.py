"""MSM parity: HIP Pippenger (gm_msm, replaces iciclegnark MsmOnDevice /
MsmG2OnDevice, icicle.go:302,315,332,355,382) vs the CPU oracle (restatement of
gnark-crypto MultiExp, prove.go:204,217,237,247,293).  Bit-exact on the affine
result (the affine form of a group element is unique)."""
import json
import os

import numpy as np
import pytest

import pyref

pytestmark = pytest.mark.gpu

CASES = [("bn254", False), ("bn254", True), ("bls12377", False), ("bls12377", True)]


def _edge_inputs(cname, g2, n, seed):
    c = pyref.CURVES[cname]
    G = pyref.Group(c, g2)
    pts = pyref.random_points(c, n, seed, g2)
    sc = pyref.random_scalars(c, n, seed + 1)
    # edge cases the reference meets: infinity (0,0) points (pk.K, icicle.go:98-105),
    # scalars 0, 1, r-1, duplicate points (DummySetup, setup.go:544-558), P and -P
    pts[1] = None
    sc[2] = 0
    sc[3] = 1
    sc[4] = c.r - 1
    pts[6] = pts[5]
    sc[6] = sc[5]
    pts[8] = G.neg(pts[7])
    sc[8] = sc[7]
    pts[10] = pts[9]
    sc[10] = c.r - sc[9]
    return sc, pts


@pytest.mark.parametrize("cname,g2", CASES)
def test_msm_small_vs_pyref(gm_ctx, cname, g2):
    c = pyref.CURVES[cname]
    n = 48
    sc, pts = _edge_inputs(cname, g2, n, 1000 + 7 * g2)
    exp = pyref.Group(c, g2).msm(sc, pts)
    sb = b"".join(pyref.encode_fr(c, s) for s in sc)
    pb = b"".join(pyref.encode_point(c, p, g2) for p in pts)
    S = gm_ctx.copy_to_device(sb)
    P = gm_ctx.copy_points_to_device(cname, pb, g2)
    for window in (0, 4, 9, 16):  # each window size gives a different sort geometry (F, NC)
        gm_ctx.set_msm_window(window)
        jac, aff = gm_ctx.msm(cname, S, P, n, g2)
        assert pyref.decode_point(c, aff, g2) == exp, (cname, g2, window)
    gm_ctx.set_msm_window(0)
    S.free()
    P.free()


@pytest.mark.parametrize("window", [0, 16])
@pytest.mark.parametrize("cname,g2", CASES)
def test_msm_empty_and_single(gm_ctx, cname, g2, window):
    import gnark_mi355x as gm
    c = pyref.CURVES[cname]
    P0 = pyref.random_points(c, 1, 5, g2)[0]
    S = gm_ctx.copy_to_device(pyref.encode_fr(c, 12345))
    P = gm_ctx.copy_points_to_device(cname, pyref.encode_point(c, P0, g2), g2)
    gm_ctx.set_msm_window(window)
    try:
        _, aff = gm_ctx.msm(cname, S, P, 0, g2)
        assert aff == bytes(gm.point_bytes(cname, g2))  # empty MSM = infinity
        _, aff = gm_ctx.msm(cname, S, P, 1, g2)
        assert pyref.decode_point(c, aff, g2) == pyref.Group(c, g2).mul(P0, 12345)
    finally:
        gm_ctx.set_msm_window(0)
        S.free()
        P.free()


@pytest.mark.parametrize("value", [0, 1, "r-1"])
@pytest.mark.parametrize("cname,g2", [("bn254", False), ("bls12377", True)])
def test_msm_constant_scalars_c16(gm_ctx, oracle, cname, g2, value):
    """All scalars equal at c = 16: 0 (every digit is zero -- nothing enters the
    sort, all buckets empty), 1 (one bucket, all others empty) and r-1 (every
    window's top digit)."""
    import gnark_mi355x as gm
    c = pyref.CURVES[cname]
    n = (1 << 14) + 3
    v = c.r - 1 if value == "r-1" else value
    sb = pyref.encode_fr(c, v) * n
    pb = _random_points_host(gm_ctx, cname, g2, n, 0x77 + g2)
    S = gm_ctx.copy_to_device(sb)
    P = gm_ctx.copy_to_device(pb)
    exp = oracle.msm(cname, g2, sb, pb)
    try:
        for window in (16, 0):
            gm_ctx.set_msm_window(window)
            assert gm_ctx.msm(cname, S, P, n, g2)[1] == exp, window
    finally:
        gm_ctx.set_msm_window(0)
        S.free()
        P.free()


def _random_points_host(ctx, cname, g2, n, seed):
    import gnark_mi355x as gm
    K = ctx.random_scalars(cname, n, seed)
    P = ctx.batch_mul_base(cname, g2, gm.generator(cname, g2), K, n)
    out = P.to_host()
    K.free()
    P.free()
    return out


def test_msm_all_equal_points(gm_ctx, oracle):
    """DummySetup shape (setup.go:544-558): every point identical -> every bucket
    add is a doubling."""
    c = pyref.BN254
    n = 4096
    P0 = pyref.random_points(c, 1, 77)[0]
    pb = pyref.encode_point(c, P0, False) * n
    sc = pyref.random_scalars(c, n, 78)
    sb = b"".join(pyref.encode_fr(c, s) for s in sc)
    S = gm_ctx.copy_to_device(sb)
    P = gm_ctx.copy_points_to_device("bn254", pb)
    _, aff = gm_ctx.msm("bn254", S, P, n)
    assert aff == oracle.msm("bn254", False, sb, pb)
    S.free()
    P.free()


@pytest.mark.parametrize("cname,g2,logn", [("bn254", False, 16), ("bn254", True, 13),
                                           ("bls12377", False, 14), ("bls12377", True, 12)])
def test_msm_random_vs_oracle(gm_ctx, oracle, cname, g2, logn):
    import gnark_mi355x as gm
    n = (1 << logn) + 37  # ragged size
    S = gm_ctx.random_scalars(cname, n, seed=0x5EED0002 + logn)
    K = gm_ctx.random_scalars(cname, n, seed=0x5EED1002 + logn)
    P = gm_ctx.batch_mul_base(cname, g2, gm.generator(cname, g2), K, n)
    sb = S.to_host()
    pb = P.to_host()
    _, aff = gm_ctx.msm(cname, S, P, n, g2)
    assert aff == oracle.msm(cname, g2, sb, pb)
    for b in (S, K, P):
        b.free()


def test_batch_mul_base_matches_oracle(gm_ctx, oracle):
    import gnark_mi355x as gm
    for cname in ("bn254", "bls12377"):
        for g2 in (False, True):
            K = gm_ctx.random_scalars(cname, 64, seed=99)
            P = gm_ctx.batch_mul_base(cname, g2, gm.generator(cname, g2), K, 64)
            assert P.to_host() == oracle.batch_mul_base(cname, g2, gm.generator(cname, g2), K.to_host())
            K.free()
            P.free()


def test_msm_skewed_scalars(gm_ctx, oracle):
    """Groth16 wire values are skewed (many 0/1/small values): one huge bucket."""
    c = pyref.BN254
    n = 1 << 14
    rng = np.random.default_rng(5)
    vals = [int(x) for x in rng.integers(0, 3, n)]
    vals[::97] = [int(x) for x in rng.integers(0, 2**62, len(vals[::97]))]
    sb = b"".join(pyref.encode_fr(c, v) for v in vals)
    import gnark_mi355x as gm
    K = gm_ctx.random_scalars("bn254", n, seed=3)
    P = gm_ctx.batch_mul_base("bn254", False, gm.generator("bn254"), K, n)
    S = gm_ctx.copy_to_device(sb)
    _, aff = gm_ctx.msm("bn254", S, P, n)
    assert aff == oracle.msm("bn254", False, sb, P.to_host())
    for b in (S, K, P):
        b.free()


@pytest.mark.parametrize("cname,g2,logn", [("bn254", False, 20), ("bn254", True, 18), ("bls12377", False, 20)])
def test_msm_huge_buckets_large(gm_ctx, oracle, cname, g2, logn):
    """Buckets spanning thousands of accumulation slices (tree-reduced fixup):
    wire-like scalars in {0, 1, 2, r-1} plus 1% random; the bls12377 case also
    has the nearly empty top window of a 253-bit field."""
    import gnark_mi355x as gm
    c = pyref.CURVES[cname]
    n = 1 << logn
    rng = np.random.default_rng(logn)
    table = np.frombuffer(b"".join(pyref.encode_fr(c, v) for v in (0, 1, 2, c.r - 1)), np.uint8).reshape(4, 32)
    sb = table[rng.integers(0, 4, n)].copy()
    R = gm_ctx.random_scalars(cname, n // 100, seed=logn)
    sb[:: 100][: n // 100] = np.frombuffer(R.to_host(), np.uint8).reshape(-1, 32)[: len(sb[::100])]
    R.free()
    sb = sb.tobytes()
    K = gm_ctx.random_scalars(cname, n, seed=5)
    P = gm_ctx.batch_mul_base(cname, g2, gm.generator(cname, g2), K, n)
    S = gm_ctx.copy_to_device(sb)
    _, aff = gm_ctx.msm(cname, S, P, n, g2=g2)
    assert aff == oracle.msm(cname, g2, sb, P.to_host())
    for b in (S, K, P):
        b.free()


@pytest.mark.parametrize("cname", ["bls12377", "bn254"])
def test_kzg_commit_and_prepared_msm(gm_ctx, oracle, cname):
    """PLONK KZG commit (kzg.Commit over pk.Kzg.G1, backend/plonk/bls12-377/prove.go:
    1158-1168): digest of a polynomial over a prefix of a device-resident SRS."""
    import gnark_mi355x as gm
    c = pyref.CURVES[cname]
    m = 5000
    tau = pyref.random_scalars(c, 1, 11)[0]
    powers = b"".join(pyref.encode_fr(c, pow(tau, i, c.r)) for i in range(m))
    srs_host = oracle.batch_mul_base(cname, False, gm.generator(cname), powers)
    srs = gm_ctx.points_upload(cname, srs_host)
    for n in (0, 1, 17, 4096, m):
        coeffs = b"".join(pyref.encode_fr(c, v) for v in pyref.random_scalars(c, n, n + 3))
        got = gm_ctx.kzg_commit(cname, srs, coeffs)
        pb = gm.point_bytes(cname, False)
        exp = oracle.msm(cname, False, coeffs, srs_host[:pb * n]) if n else bytes(pb)
        assert got == exp, n
    with pytest.raises(gm.GmError):
        gm_ctx.kzg_commit(cname, srs, bytes(32 * (m + 1)))
    # generic prepared MSM equals the raw-buffer MSM
    S = gm_ctx.random_scalars(cname, m, seed=9)
    P = gm_ctx.copy_to_device(srs_host)
    assert gm_ctx.msm_prepared(cname, S, srs, m)[1] == gm_ctx.msm(cname, S, P, m)[1]
    for b in (S, P, srs):
        b.free()


@pytest.mark.parametrize("cname,g2", CASES)
def test_msm_precomputed_edge_vs_pyref(gm_ctx, cname, g2):
    """Fixed-base precomputed set (W window copies, one shared bucket set): the
    same edge inputs as the plain MSM, several windows, prefixes n <= prepared_n."""
    c = pyref.CURVES[cname]
    n = 48
    sc, pts = _edge_inputs(cname, g2, n, 3000 + 7 * g2)
    G = pyref.Group(c, g2)
    sb = b"".join(pyref.encode_fr(c, s) for s in sc)
    pb = b"".join(pyref.encode_point(c, p, g2) for p in pts)
    S = gm_ctx.copy_to_device(sb)
    for window in (0, 5, 9, 16):
        pre = gm_ctx.points_upload_precomputed(cname, pb, g2, window)
        for m in (n, 29, 1, 0):
            _, aff = gm_ctx.msm_precomputed(cname, S, pre, m, g2)
            exp = G.msm(sc[:m], pts[:m])
            assert pyref.decode_point(c, aff, g2) == exp, (cname, g2, window, m)
        pre.free()
    S.free()


@pytest.mark.parametrize("cname,g2,logn", [("bn254", False, 16), ("bn254", True, 12),
                                           ("bls12377", False, 14), ("bls12377", True, 11)])
def test_msm_precomputed_random_vs_oracle(gm_ctx, oracle, cname, g2, logn):
    import gnark_mi355x as gm
    n = (1 << logn) + 37
    S = gm_ctx.random_scalars(cname, n, seed=0x5EED0005 + logn)
    K = gm_ctx.random_scalars(cname, n, seed=0x5EED1005 + logn)
    P = gm_ctx.batch_mul_base(cname, g2, gm.generator(cname, g2), K, n)
    sb, pb = S.to_host(), P.to_host()
    pre = gm_ctx.points_upload_precomputed(cname, pb, g2, 0)
    _, aff = gm_ctx.msm_precomputed(cname, S, pre, n, g2)
    assert aff == oracle.msm(cname, g2, sb, pb)
    # skewed wire-like scalars: huge shared buckets (long-span fixup)
    c = pyref.CURVES[cname]
    rng = np.random.default_rng(logn)
    table = np.frombuffer(b"".join(pyref.encode_fr(c, v) for v in (0, 1, 2, c.r - 1)), np.uint8).reshape(4, 32)
    sk = table[rng.integers(0, 4, n)].tobytes()
    S2 = gm_ctx.copy_to_device(sk)
    _, aff = gm_ctx.msm_precomputed(cname, S2, pre, n, g2)
    assert aff == oracle.msm(cname, g2, sk, pb)
    for b in (S, S2, K, P, pre):
        b.free()


def test_msm_precomputed_large_matches_plain(gm_ctx):
    """2^20 BN254 G1 (the bench workload): precomputed == plain, bit-exact."""
    import gnark_mi355x as gm
    n = 1 << 20
    S = gm_ctx.random_scalars("bn254", n, seed=0x5EED0002)
    K = gm_ctx.random_scalars("bn254", n, seed=0x5EED1002)
    P = gm_ctx.batch_mul_base("bn254", False, gm.generator("bn254"), K, n)
    pre = gm_ctx.points_upload_precomputed("bn254", P.to_host(), False, 0)
    assert gm_ctx.msm_precomputed("bn254", S, pre, n)[1] == gm_ctx.msm("bn254", S, P, n)[1]
    for b in (S, K, P, pre):
        b.free()


@pytest.mark.parametrize("window", [0, 16])
@pytest.mark.parametrize("cname,g2", CASES)
def test_msm_bucket_chain_special_cases(gm_ctx, cname, g2, window):
    """Within one bucket the accumulator meets -(running sum) (-> infinity) and
    +(running sum) (-> doubling) after several adds, i.e. while its coordinates
    are non-canonical (lazily reduced G1 accumulation, field.hpp).  All scalars
    are 1: every point lands in bucket 1 of window 0, accumulated in index order."""
    c = pyref.CURVES[cname]
    G = pyref.Group(c, g2)
    base = pyref.random_points(c, 12, 4242 + g2, g2)
    pts, run = [], None
    for i, P in enumerate(base):
        if i in (3, 9):
            Q = G.neg(run)           # acc + (-acc) = infinity
        elif i in (6,):
            Q = run                  # acc + acc = doubling
        else:
            Q = P
        pts.append(Q)
        run = Q if run is None else G.add(run, Q)
    n = len(pts)
    sb = b"".join(pyref.encode_fr(c, 1) for _ in range(n))
    pb = b"".join(pyref.encode_point(c, p, g2) for p in pts)
    exp = G.msm([1] * n, pts)
    S = gm_ctx.copy_to_device(sb)
    P = gm_ctx.copy_points_to_device(cname, pb, g2)
    gm_ctx.set_msm_window(window)
    try:
        _, aff = gm_ctx.msm(cname, S, P, n, g2)
    finally:
        gm_ctx.set_msm_window(0)
    assert pyref.decode_point(c, aff, g2) == exp
    pre = gm_ctx.points_upload_precomputed(cname, pb, g2, window)
    _, aff = gm_ctx.msm_precomputed(cname, S, pre, n, g2)
    assert pyref.decode_point(c, aff, g2) == exp
    for b in (S, P, pre):
        b.free()


@pytest.mark.parametrize("cname,g2,logn", [("bn254", False, 14), ("bn254", True, 12),
                                           ("bls12377", False, 13), ("bls12377", True, 11)])
def test_msm_sort_geometries_vs_oracle(gm_ctx, oracle, cname, g2, logn):
    """Window sizes 8..20 give bucket counts from 2^12 to 13 * 2^19, i.e. every
    shape of the two-level bucket sort: one coarse bin covering all buckets
    (F >= log2 T), ~16K entries per coarse bin, and mostly empty buckets."""
    import gnark_mi355x as gm
    n = (1 << logn) + 11
    S = gm_ctx.random_scalars(cname, n, seed=0x5EED0007 + logn)
    K = gm_ctx.random_scalars(cname, n, seed=0x5EED1007 + logn)
    P = gm_ctx.batch_mul_base(cname, g2, gm.generator(cname, g2), K, n)
    exp = oracle.msm(cname, g2, S.to_host(), P.to_host())
    for c in (16, 15, 8, 20):
        gm_ctx.set_msm_window(c)
        try:
            assert gm_ctx.msm(cname, S, P, n, g2)[1] == exp, c
        finally:
            gm_ctx.set_msm_window(0)
    for b in (S, K, P):
        b.free()


@pytest.mark.parametrize("value", [1, 3])
def test_msm_split_coarse_bin(gm_ctx, oracle, value):
    """One bucket holding 2^19 + 5 entries (> S2_BIG = 2^18): its coarse bin is
    split into parts (k_msm_s2_scan / k_msm_s2_scatter path of the sort)."""
    import gnark_mi355x as gm
    cname = "bn254"
    c = pyref.CURVES[cname]
    n = (1 << 19) + 5
    sb = pyref.encode_fr(c, value) * n
    K = gm_ctx.random_scalars(cname, n, seed=0x5117)
    P = gm_ctx.batch_mul_base(cname, False, gm.generator(cname, False), K, n)
    S = gm_ctx.copy_to_device(sb)
    try:
        assert gm_ctx.msm(cname, S, P, n, False)[1] == oracle.msm(cname, False, sb, P.to_host())
    finally:
        for b in (S, K, P):
            b.free()


@pytest.mark.parametrize("cname,g2,window,pre", [("bn254", False, 16, False), ("bn254", False, 0, True),
                                                 ("bls12377", True, 0, False), ("bn254", True, 0, True)])
def test_msm_three_level_sort_vs_oracle(gm_ctx, oracle, monkeypatch, cname, g2, window, pre):
    """The middle pass of the bucket sort (pass-1 super-bins split into coarse
    bins, msm_sort.hip) runs by itself only for large MSMs (2^22+, precomputed
    2^20+); GM_MSM_SORT_MING forces it here, at several depths."""
    import gnark_mi355x as gm
    n = (1 << 14) + 11
    S = gm_ctx.random_scalars(cname, n, seed=0x3EED0007)
    K = gm_ctx.random_scalars(cname, n, seed=0x3EED1007)
    P = gm_ctx.batch_mul_base(cname, g2, gm.generator(cname, g2), K, n)
    exp = oracle.msm(cname, g2, S.to_host(), P.to_host())
    pts = gm_ctx.points_upload_precomputed(cname, P.to_host(), g2, window) if pre else None
    try:
        for ming in (1, 3, 6):
            monkeypatch.setenv("GM_MSM_SORT_MING", str(ming))
            gm_ctx.set_msm_window(0 if pre else window)
            if pre:
                got = gm_ctx.msm_precomputed(cname, S, pts, n, g2)[1]
            else:
                got = gm_ctx.msm(cname, S, P, n, g2)[1]
            assert got == exp, ming
    finally:
        gm_ctx.set_msm_window(0)
        for b in (S, K, P) + ((pts,) if pre else ()):
            b.free()


def test_msm_three_level_sort_skewed(gm_ctx, oracle, monkeypatch):
    """Middle pass + split final bins: one bucket of 2^19 + 5 entries."""
    import gnark_mi355x as gm
    monkeypatch.setenv("GM_MSM_SORT_MING", "2")
    c = pyref.CURVES["bn254"]
    n = (1 << 19) + 5
    sb = pyref.encode_fr(c, 2) * n
    K = gm_ctx.random_scalars("bn254", n, seed=0x5118)
    P = gm_ctx.batch_mul_base("bn254", False, gm.generator("bn254", False), K, n)
    S = gm_ctx.copy_to_device(sb)
    try:
        assert gm_ctx.msm("bn254", S, P, n, False)[1] == oracle.msm("bn254", False, sb, P.to_host())
    finally:
        for b in (S, K, P):
            b.free()


def test_msm_async_pipelined(gm_ctx, oracle):
    """gm_msm_async / gm_msm_wait: MSMs in flight (different curves, groups and
    sizes), waited in order, equal the oracle; three may be in flight, a fourth
    is refused."""
    import gnark_mi355x as gm
    cases = []
    for cname, g2, n in (("bn254", False, 5000), ("bls12377", True, 777), ("bn254", True, 3000)):
        S = gm_ctx.random_scalars(cname, n, seed=0xA5A5 + n)
        K = gm_ctx.random_scalars(cname, n, seed=0x5A5A + n)
        P = gm_ctx.batch_mul_base(cname, g2, gm.generator(cname, g2), K, n)
        K.free()
        cases.append((cname, g2, n, S, P, oracle.msm(cname, g2, S.to_host(), P.to_host())))
    try:
        pend = []
        for k, (cname, g2, n, S, P, exp) in enumerate(cases):
            pend.append(gm_ctx.msm_async(cname, S, P, n, g2))
            if k >= 1:
                assert pend[k - 1].wait()[1] == cases[k - 1][5]
        assert pend[-1].wait()[1] == cases[-1][5]
        a = gm_ctx.msm_async("bn254", cases[0][3], cases[0][4], cases[0][2])
        b = gm_ctx.msm_async(cases[1][0], cases[1][3], cases[1][4], cases[1][2], cases[1][1])
        c = gm_ctx.msm_async("bn254", cases[0][3], cases[0][4], cases[0][2])
        with pytest.raises(gm.GmError, match="in flight"):
            gm_ctx.msm_async("bn254", cases[0][3], cases[0][4], cases[0][2])
        assert a.wait()[1] == cases[0][5] and b.wait()[1] == cases[1][5] and c.wait()[1] == cases[0][5]
    finally:
        for c in cases:
            c[3].free()
            c[4].free()


def test_msm_accum_wave_stamps(gm_ctx, oracle):
    """Profiled G1 MSMs (sync and async) record the accumulation's first-wave ..
    last-wave execution (msm_accum_g1_exec, the bench roofline's kernel time) next
    to its launch event brackets (msm_accum_g1): one stamp per launch, inside the
    bracket; the results stay the oracle's."""
    import gnark_mi355x as gm
    n = 1 << 14
    S = gm_ctx.random_scalars("bn254", n, seed=0x57A3)
    K = gm_ctx.random_scalars("bn254", n, seed=0x57A4)
    P = gm_ctx.batch_mul_base("bn254", False, gm.generator("bn254", False), K, n)
    K.free()
    try:
        exp = oracle.msm("bn254", False, S.to_host(), P.to_host())
        gm_ctx.profile_reset()
        gm_ctx.profile(True)
        assert gm_ctx.msm("bn254", S, P, n)[1] == exp
        pend = [gm_ctx.msm_async("bn254", S, P, n) for _ in range(3)]
        assert all(p.wait()[1] == exp for p in pend)
        gm_ctx.profile(False)
        st = gm_ctx.profile_stats()
        ex_ms, ex_cnt = st["msm_accum_g1_exec"]
        br_ms, br_cnt = st["msm_accum_g1"]
        assert ex_cnt == br_cnt == 4
        assert 0 < ex_ms <= br_ms * 1.02 + 0.01
        gm_ctx.profile_reset()
        assert "msm_accum_g1_exec" not in gm_ctx.profile_stats()
    finally:
        gm_ctx.profile(False)
        S.free()
        P.free()


def test_msm_async_interleaved_with_sync(gm_ctx, oracle):
    """Synchronous MSMs (small and large: a large one also takes a readback
    buffer for its max-span check) issued while two async MSMs are pending must
    not reuse the pending MSMs' pinned readback buffers (gnark_mi355x.h: each
    pending MSM keeps its own until gm_msm_wait)."""
    import gnark_mi355x as gm
    sizes = [(3000, False), (1 << 18, False), (700, True), (5000, False), (1 << 18, False), (900, True)]
    data = []
    for k, (n, g2) in enumerate(sizes):
        S = gm_ctx.random_scalars("bn254", n, seed=0xC0 + k)
        K = gm_ctx.random_scalars("bn254", n, seed=0xD0 + k)
        P = gm_ctx.batch_mul_base("bn254", g2, gm.generator("bn254", g2), K, n)
        K.free()
        data.append((n, g2, S, P, oracle.msm("bn254", g2, S.to_host(), P.to_host())))
    try:
        a = gm_ctx.msm_async("bn254", data[0][2], data[0][3], data[0][0], data[0][1])
        b = gm_ctx.msm_async("bn254", data[2][2], data[2][3], data[2][0], data[2][1])
        for n, g2, S, P, exp in data[1:] + data[1:]:  # 10 synchronous MSMs in between
            assert gm_ctx.msm("bn254", S, P, n, g2)[1] == exp
        assert a.wait()[1] == data[0][4]
        assert b.wait()[1] == data[2][4]
    finally:
        for d in data:
            d[2].free()
            d[3].free()


def test_msm_async_after_queued_producer(gm_ctx, oracle):
    """gm_msm_async orders its MSM after the work already queued on the context
    stream (a marker only when that stream is busy, csrc/capi.hip): the scalars
    are produced by an in-place NTT and the points by a d2d copy queued right
    before each async MSM, with no synchronisation in between, and three MSMs
    run pipelined; every result is the oracle's MSM of the produced inputs."""
    import gnark_mi355x as gm
    n = 1 << 18
    S0 = gm_ctx.random_scalars("bn254", n, seed=0x71)
    K = gm_ctx.random_scalars("bn254", n, seed=0x72)
    P0 = gm_ctx.batch_mul_base("bn254", False, gm.generator("bn254"), K, n)
    K.free()
    s_host, p_host = S0.to_host(), P0.to_host()
    exp = oracle.msm("bn254", False, oracle.fft("bn254", s_host, 0, 0, 0), p_host)
    bufs = [(gm_ctx.malloc(32 * n), gm_ctx.malloc(64 * n)) for _ in range(3)]
    try:
        pend = []
        for S, P in bufs:
            S.copy_from(S0)
            gm_ctx.ntt("bn254", S, n, False, False, False)
            P.copy_from(P0)
            pend.append(gm_ctx.msm_async("bn254", S, P, n))
        assert [p.wait()[1] for p in pend] == [exp] * 3
    finally:
        for S, P in bufs:
            S.free()
            P.free()
        S0.free()
        P0.free()


def test_msm_async_inputs_overwritten_in_place(gm_ctx, oracle):
    """A synchronous call queued after gm_msm_async may overwrite the pending
    MSM's scalars and points in place (include/gnark_mi355x.h): the context
    stream waits until the MSM has read them (after its digits and point
    conversion), while the accumulation and reduction still run on the MSM's
    own stream.  Here an in-place gm_ntt over the scalars and a d2d copy over the
    points follow each of two pending 2^20 MSMs at once; both results are the
    oracle's MSM of the ORIGINAL inputs, and the overwrites did happen."""
    import gnark_mi355x as gm
    n = 1 << 20
    ins = []
    for k in range(2):
        S = gm_ctx.random_scalars("bn254", n, seed=0xE0 + k)
        K = gm_ctx.random_scalars("bn254", n, seed=0xF0 + k)
        P = gm_ctx.batch_mul_base("bn254", False, gm.generator("bn254"), K, n)
        ins.append((S, P, K, S.to_host(), P.to_host()))
    try:
        exp = [oracle.msm("bn254", False, sh, ph) for _, _, _, sh, ph in ins]
        junk = gm_ctx.random_scalars("bn254", 2 * n, seed=0xAB)  # 64 B per point of junk
        pend = []
        for S, P, K, sh, ph in ins:
            pend.append(gm_ctx.msm_async("bn254", S, P, n))
            gm_ctx.ntt("bn254", S, n, False, False, False)          # scalars overwritten in place
            gm.load_library().gm_memcpy_d2d(gm_ctx.handle, P.ptr, junk.ptr, 64 * n)  # points overwritten
        got = [p.wait()[1] for p in pend]
        assert got == exp
        assert ins[0][0].to_host() == oracle.fft("bn254", ins[0][3], 0, 0, 0)
        assert ins[1][1].to_host() == junk.to_host()
        junk.free()
    finally:
        for S, P, K, _, _ in ins:
            for b in (S, P, K):
                b.free()


def test_gm_destroy_with_msms_pending(oracle):
    """gm_destroy with two gm_msm_async MSMs pending: it waits for their device
    work and releases their slot arenas and readback buffers before freeing the
    context (capi.hip gm_destroy / orphan_pending_msms); each handle's
    gm_msm_wait then reports the destroyed context and frees the handle.  The
    inputs may be freed while the MSMs are pending (they have been read once the
    context stream is past gm_msm_async).  A fresh context afterwards works."""
    import gnark_mi355x as gm
    n = 1 << 18
    ctx = gm.Context(0)
    S = ctx.random_scalars("bn254", n, seed=0x77)
    K = ctx.random_scalars("bn254", n, seed=0x78)
    P = ctx.batch_mul_base("bn254", False, gm.generator("bn254"), K, n)
    K.free()
    a = ctx.msm_async("bn254", S, P, n)
    b = ctx.msm_async("bn254", S, P, n, False)
    S.free()
    P.free()
    ctx.close()
    for p in (a, b):
        with pytest.raises(gm.GmError, match="destroyed"):
            p.wait()
    with gm.Context(0) as c2:
        S = c2.random_scalars("bn254", 3000, seed=0x79)
        K = c2.random_scalars("bn254", 3000, seed=0x7A)
        P = c2.batch_mul_base("bn254", False, gm.generator("bn254"), K, 3000)
        pend = c2.msm_async("bn254", S, P, 3000)
        assert pend.wait()[1] == oracle.msm("bn254", False, S.to_host(), P.to_host())
        for x in (S, K, P):
            x.free()


def _glv_bls12377():
    import importlib.util
    spec = importlib.util.spec_from_file_location(
        "glv_constants", os.path.join(os.path.dirname(__file__), "..", "tools", "glv_constants.py"))
    glv = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(glv)
    return glv.derive_bls12377()


@pytest.mark.parametrize("g2,window", [(False, 0), (False, 13), (True, 0), (True, 16)])
def test_msm_glv_bls12377_split_boundaries(gm_ctx, oracle, g2, window):
    """BLS12-377 GLV (msm_impl.hpp GlvBls377: k2 = floor(k / lambda), k1 = k mod
    lambda, lambda = x^2 - 1; phi = (beta x, y), beta^2 on the G2 twist): scalars
    at the division's edges against the oracle's unsplit Pippenger, with the
    split on and off."""
    c = pyref.CURVES["bls12377"]
    d = _glv_bls12377()
    r, lam = c.r, d["lam"]
    special = [0, 1, 2, r - 1, r - 2, lam, lam - 1, lam + 1, lam * lam, lam * lam - 1, lam * lam + lam,
               lam * lam + lam - 1, r - lam, (r - 1) // 2, 1 << 252, (1 << 127) - 1, 1 << 127, 2 * lam]
    n = 2048 + 21 if not g2 else 512 + 21
    pbytes = 192 if g2 else 96
    sc = pyref.random_scalars(c, n, 0x71F + g2)
    sc[:len(special)] = special
    sb = b"".join(pyref.encode_fr(c, s) for s in sc)
    pb = _random_points_host(gm_ctx, "bls12377", g2, n, 0x720 + g2)
    pb = pyref.encode_point(c, None, g2) + pb[pbytes:]  # an infinity point
    S = gm_ctx.copy_to_device(sb)
    P = gm_ctx.copy_to_device(pb)
    exp = oracle.msm("bls12377", g2, sb, pb)
    try:
        gm_ctx.set_msm_window(window)
        for glv in (1, 0):
            gm_ctx.set_msm_glv(glv)
            for m in (1, 9, 64, n):
                exp_m = exp if m == n else oracle.msm("bls12377", g2, sb[:32 * m], pb[:pbytes * m])
                assert gm_ctx.msm("bls12377", S, P, m, g2)[1] == exp_m, (g2, window, glv, m)
    finally:
        gm_ctx.set_msm_window(0)
        gm_ctx.set_msm_glv(-1)
        S.free()
        P.free()


@pytest.mark.parametrize("glv", [1, 0])
def test_msm_bn254_g1_2p20_bench_input_vs_oracle(gm_ctx, oracle, glv):
    """BASELINE configs[1] at full size, exactly the bench's input (bench.py:
    uniform scalars seed 0x5EED0002, points [k_i]G1 seed 0x5EED1002, plus the
    edge set -- 1% infinity points, a 1% run of equal points, scalars 0, 1, r-1),
    GLV split on (the default path) and off, against the oracle's Pippenger."""
    import importlib.util
    import gnark_mi355x as gm
    spec = importlib.util.spec_from_file_location("bench", os.path.join(os.path.dirname(__file__), "..", "bench.py"))
    bench = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(bench)
    n = 1 << 20
    S = gm_ctx.random_scalars("bn254", n, 0x5EED0002)
    K = gm_ctx.random_scalars("bn254", n, 0x5EED1002)
    P = gm_ctx.batch_mul_base("bn254", False, gm.generator("bn254"), K, n)
    K.free()
    try:
        bench.add_edge_set(gm_ctx, gm, S, P, n)
        exp = oracle.msm("bn254", False, S.to_host(), P.to_host())
        gm_ctx.set_msm_glv(glv)
        assert gm_ctx.msm("bn254", S, P, n)[1] == exp
        pend = [gm_ctx.msm_async("bn254", S, P, n) for _ in range(2)]  # the bench's pipelined form
        assert [q.wait()[1] for q in pend] == [exp, exp]
    finally:
        gm_ctx.set_msm_glv(-1)
        S.free()
        P.free()


@pytest.mark.parametrize("g2,window", [(False, 0), (False, 11), (False, 16), (True, 0), (True, 16)])
def test_msm_glv_split_boundaries(gm_ctx, oracle, g2, window):
    """BN254 G1 / G2 MSMs from gnark-layout points run the GLV split (k = k1 + k2
    lambda, |k1|, |k2| < 2^127, points P_i and phi(P_i) = (beta x, y), beta^2 on
    the G2 twist; msm_impl.hpp GlvBn254): scalars at the split's edges -- lambda,
    r - lambda, the basis entries, k2 of both signs, r - 1 -- plus random ones,
    against the oracle's unsplit Pippenger."""
    c = pyref.BN254
    import importlib.util
    spec = importlib.util.spec_from_file_location(
        "glv_constants", os.path.join(os.path.dirname(__file__), "..", "tools", "glv_constants.py"))
    glv = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(glv)
    d = glv.derive()
    r, lam = c.r, d["lam"]
    special = [0, 1, 2, r - 1, r - 2, lam, r - lam, lam + 1, lam - 1, d["a1"], d["b2"], r - d["b2"],
               d["a2"], r - d["a2"], (r - 1) // 2, (r + 1) // 2, 1 << 253, (1 << 127) - 1, 1 << 127]
    n = 4096 + 19 if not g2 else 1024 + 19
    pbytes = 128 if g2 else 64
    sc = pyref.random_scalars(c, n, 0x61F)
    sc[:len(special)] = special
    sb = b"".join(pyref.encode_fr(c, s) for s in sc)
    pb = _random_points_host(gm_ctx, "bn254", g2, n, 0x620)
    pb = pyref.encode_point(c, None, g2) + pb[pbytes:]  # an infinity point
    S = gm_ctx.copy_to_device(sb)
    P = gm_ctx.copy_to_device(pb)
    exp = oracle.msm("bn254", g2, sb, pb)
    try:
        gm_ctx.set_msm_window(window)
        for m in (1, 7, 64, n):
            exp_m = exp if m == n else oracle.msm("bn254", g2, sb[:32 * m], pb[:pbytes * m])
            assert gm_ctx.msm("bn254", S, P, m, g2)[1] == exp_m, (g2, window, m)
    finally:
        gm_ctx.set_msm_window(0)
        S.free()
        P.free()
