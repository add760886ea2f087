"""BASELINE.json configs at their full sizes, checked against the CPU oracle.

  configs[2]  BN254 Fr NTT+INTT 2^24 (all 8 fft.Domain modes, prove.go:372-378,396)
              + the full Groth16 prove at 2^20 R1CS end-to-end from HOST inputs
              (gm_g16_prove; icicle.go:133-422 / prove.go:62-325), byte-identical
              to the oracle prover and accepted by the exponent check.
  configs[3]  BN254 Groth16 prove at 2^24 on one GPU (synthetic pk, plain and
              precomputed) and the sharded data path (gm_g16_pk_upload_shard /
              gm_g16_prove_partial / gm_g16_finish) at world = 8, n = 2^20.
  configs[4]  BLS12-377 G1 and G2 MSM at 2^22 (icicle.go:302-382 / prove.go:204-293).

The oracle (oracle/gm_oracle.cpp, a restatement of gnark-crypto) runs on the
host's cores; parity is "unpinned" at the gnark-crypto boundary.
"""
import os
import time

import numpy as np
import pytest

import pyref
import r1cs as R

pytestmark = pytest.mark.gpu

MODES = [(i, d, c) for i in (0, 1) for d in (0, 1) for c in (0, 1)]  # inverse, dit, coset
TOXIC = [0x1D5A2B3C4D5E6F708192A3B4C5D6E7F8091A2B3C4D5E6F708192A3B4C5D6E7,
         0x2E6B3C4D5E6F708192A3B4C5D6E7F8091A2B3C4D5E6F708192A3B4C5D6E7F8,
         0x3F7C4D5E6F708192A3B4C5D6E7F8091A2B3C4D5E6F708192A3B4C5D6E7F809,
         0x0A8D5E6F708192A3B4C5D6E7F8091A2B3C4D5E6F708192A3B4C5D6E7F8091A,
         0x1B9E6F708192A3B4C5D6E7F8091A2B3C4D5E6F708192A3B4C5D6E7F8091A2B]


def _log(msg):
    # progress on stdout (pytest -s): these tests run minutes of oracle work
    print("  [%s] %s" % (time.strftime("%H:%M:%S"), msg), flush=True)


def _random_points(ctx, curve, g2, n, seed):
    """n points [k_i]G with seeded random k_i (gnark affine bytes, host)."""
    import gnark_mi355x as gm
    K = ctx.random_scalars(curve, n, seed)
    P = ctx.batch_mul_base(curve, g2, gm.generator(curve, g2), K, n)
    out = np.frombuffer(P.to_host(), np.uint8)
    K.free()
    P.free()
    return out


def test_ntt_2p24_all_modes_vs_oracle(gm_ctx, oracle):
    """configs[2]: every (inverse, DIF/DIT, coset) mode of the 2^24 transform."""
    n = 1 << 24
    X = gm_ctx.random_scalars("bn254", n, seed=0x5EED0003)
    xb = X.to_host()
    try:
        for inverse, dit, coset in MODES:
            X.write(xb)
            gm_ctx.ntt("bn254", X, n, inverse, dit, coset)
            assert X.to_host() == oracle.fft("bn254", xb, inverse, dit, coset), (inverse, dit, coset)
            _log("ntt 2^24 mode %s ok" % ((inverse, dit, coset),))
    finally:
        X.free()


@pytest.fixture(scope="module")
def chain_2p20(oracle):
    """refCircuit (groth16_test.go:120-156) with 2^20 - 1 squarings: nc = 2^20
    constraints, n = 2^20; a real (toxic-waste) setup by the oracle."""
    cname = "bn254"
    c = pyref.CURVES[cname]
    r1, W, a, b, cc = R.squaring_chain_fast((1 << 20) - 1, cname, x=2)
    assert r1.domain_size == 1 << 20
    tox = R.encode_vec(cname, [t % c.r for t in TOXIC])
    _log("chain 2^20 built; oracle setup")
    pk = oracle.g16_setup(cname, r1, tox)
    rb, sb = R.encode_vec(cname, [0xC0FFEE1234]), R.encode_vec(cname, [0xBADC0DE5678])
    _log("oracle prove")
    exp = oracle.g16_prove(cname, pk, r1.nb_public, W, a, b, cc, rb, sb)
    _log("oracle check")
    assert oracle.g16_check(cname, r1, tox, W, rb, sb, *exp) == 7
    _log("oracle proof verified")
    return dict(cname=cname, r1=r1, W=W, a=a, b=b, c=cc, tox=tox, pk=pk, r=rb, s=sb, exp=exp)


@pytest.mark.parametrize("precompute", [False, True])
def test_groth16_2p20_host_inputs(gm_ctx, oracle, chain_2p20, precompute):
    """configs[2]: full prove at 2^20 through gm_g16_prove with host-resident
    wires / a / b / c (the icicle.go:204-412 scope incl. its H2D copies)."""
    import gnark_mi355x as gm
    d = chain_2p20
    r1 = d["r1"]
    dpk = gm.ProvingKey(gm_ctx, d["cname"], d["pk"], r1.domain_size, r1.nb_wires, r1.nb_public,
                        precompute=precompute)
    try:
        got = dpk.prove(d["W"], d["a"], d["b"], d["c"], d["r"], d["s"])
    finally:
        dpk.free()
    assert got == d["exp"]
    assert oracle.g16_check(d["cname"], r1, d["tox"], d["W"], d["r"], d["s"], *got) == 7


def test_groth16_2p20_sharded_world8(gm_ctx, chain_2p20):
    """configs[3] data path at world = 8 on one GPU: each rank's pk slice and
    partial sums in turn, summed and finished on the host."""
    import gnark_mi355x as gm
    d = chain_2p20
    r1 = d["r1"]
    n, world = r1.domain_size, 8
    parts = []
    W = gm_ctx.copy_to_device(d["W"])
    try:
        for rank in range(world):
            dpk = gm.ProvingKey(gm_ctx, d["cname"], d["pk"], n, r1.nb_wires, r1.nb_public, precompute=(rank % 2 == 1),
                                shard=(rank, world))
            abc = []
            try:
                for v in (d["a"], d["b"], d["c"]):
                    buf = gm_ctx.malloc(32 * n)
                    buf.write(bytes(32 * n))
                    buf.write(v)
                    abc.append(buf)
                parts.append(dpk.prove_partial_device(W, *abc, r1.nc))
            finally:
                for x in abc:
                    x.free()
                if rank < world - 1:
                    dpk.free()
        got = gm.g16_finish(d["cname"], dpk._h, gm.g16_reduce_partials(d["cname"], parts), d["r"], d["s"])
        dpk.free()
    finally:
        W.free()
    assert got == d["exp"]


@pytest.mark.parametrize("ndev,precompute", [(4, False), (3, True)])
def test_groth16_2p20_multi_contexts(chain_2p20, ndev, precompute):
    """Single-process multi-device prove (gm_g16_prove_multi) with `ndev`
    contexts on the one test GPU: sharded key (device 0 lighter), wire slices,
    computeH on device 0, h slices copied to the others, host-summed partials."""
    import gnark_mi355x as gm
    d = chain_2p20
    r1 = d["r1"]
    with gm.Multi([0] * ndev) as m:
        mpk = gm.ProvingKeyMulti(m, d["cname"], d["pk"], r1.domain_size, r1.nb_wires, r1.nb_public,
                                 precompute=precompute)
        try:
            got = mpk.prove(d["W"], d["a"], d["b"], d["c"], d["r"], d["s"])
        finally:
            mpk.free()
    assert got == d["exp"]


@pytest.mark.parametrize("g2", [False, True])
def test_msm_bls12377_2p22_vs_oracle(gm_ctx, oracle, g2):
    """configs[4]: BLS12-377 G1 / G2 MSM at 2^22, uniform scalars, random points."""
    n = 1 << 22
    S = gm_ctx.random_scalars("bls12377", n, seed=0x5EED0004 + g2)
    pb = _random_points(gm_ctx, "bls12377", g2, n, 0x5EED1004 + g2)
    P = gm_ctx.copy_to_device(pb)
    try:
        _, aff = gm_ctx.msm("bls12377", S, P, n, g2=g2)
        _log("gpu msm done; oracle msm")
        assert aff == oracle.msm("bls12377", g2, S.to_host(), pb)
    finally:
        S.free()
        P.free()


def test_groth16_2p24_synthetic_pk(gm_ctx, oracle):
    """configs[3] on one GPU: n = 2^24 Groth16 prove (host inputs) over a
    synthetic proving key of random points (a setup at 2^24 is out of the
    oracle's time budget), plain and precomputed device keys, byte-identical to
    the oracle prover on the same key and inputs."""
    import gnark_mi355x as gm
    cname = "bn254"
    n = 1 << 24
    nb_public = 2
    nb_wires = n + 2
    nc = n - 3  # ragged: a, b, c shorter than the domain (zero-padded, prove.go:364-370)
    g1b = gm.point_bytes(cname, False)
    small1 = _random_points(gm_ctx, cname, False, 3, 101)
    small2 = _random_points(gm_ctx, cname, True, 2, 102)
    infA = np.zeros(nb_wires, np.uint8)
    infB = np.zeros(nb_wires, np.uint8)
    infA[[5, 77, 1000]] = 1  # wires whose A(t) / B(t) are 0: dropped by the compaction
    infB[[6, 78]] = 1
    pk = {"g1_alpha": small1[:g1b], "g1_beta": small1[g1b:2 * g1b], "g1_delta": small1[2 * g1b:],
          "g1_A": _random_points(gm_ctx, cname, False, nb_wires - 3, 103),
          "g1_B": _random_points(gm_ctx, cname, False, nb_wires - 2, 104),
          "g1_Z": _random_points(gm_ctx, cname, False, n - 1, 105),
          "g1_K": _random_points(gm_ctx, cname, False, nb_wires - nb_public, 106),
          "g2_beta": small2[:2 * g1b], "g2_delta": small2[2 * g1b:],
          "g2_B": _random_points(gm_ctx, cname, True, nb_wires - 2, 107),
          "infA": infA, "infB": infB}
    pk["sizes"] = np.array([n, nb_wires, nb_wires - 3, nb_wires - 2, nb_wires - nb_public], np.uint64)
    bufs = [gm_ctx.random_scalars(cname, m, 110 + i) for i, m in enumerate((nb_wires, nc, nc, nc))]
    W, a, b, cc = (x.to_host() for x in bufs)
    for x in bufs:
        x.free()
    rb, sb = R.encode_vec(cname, [0x123456789]), R.encode_vec(cname, [0x987654321])
    _log("synthetic 2^24 pk ready; oracle prove")
    exp = oracle.g16_prove(cname, pk, nb_public, W, a, b, cc, rb, sb)
    _log("oracle prove done")
    for precompute in (False, True):
        dpk = gm.ProvingKey(gm_ctx, cname, {k: v for k, v in pk.items() if k != "sizes"}, n, nb_wires, nb_public,
                            precompute=precompute)
        try:
            got = dpk.prove(W, a, b, cc, rb, sb)
        finally:
            dpk.free()
        assert got == exp, precompute
        _log("gpu prove (precompute=%s) matches" % precompute)
    # configs[3]'s own form: the same 2^24 key as world = 8 shards (one GPU
    # plays every rank in turn): each rank's slice (gm_g16_pk_upload_shard),
    # its five partial sums (gm_g16_prove_partial), host-reduced and finished
    # (gm_g16_finish) -- byte-identical to the same oracle proof
    world = 8
    dev = [gm_ctx.copy_to_device(W)] + [gm_ctx.malloc(32 * n) for _ in range(3)]
    parts = []
    hpk = {k: v for k, v in pk.items() if k != "sizes"}
    try:
        for rank in range(world):
            dpk = gm.ProvingKey(gm_ctx, cname, hpk, n, nb_wires, nb_public, precompute=(rank % 2 == 1),
                                shard=(rank, world))
            try:
                for buf, v in zip(dev[1:], (a, b, cc)):  # computeH overwrites a, b, c: fresh per rank
                    buf.write(bytes(32 * n))
                    buf.write(v)
                parts.append(dpk.prove_partial_device(dev[0], dev[1], dev[2], dev[3], nc))
                if rank == world - 1:
                    got = gm.g16_finish(cname, dpk._h, gm.g16_reduce_partials(cname, parts), rb, sb)
            finally:
                dpk.free()
    finally:
        for x in dev:
            x.free()
    assert got == exp
    _log("sharded world=8 prove matches")


@pytest.mark.skipif(os.environ.get("GM_TEST_CONFIG4_FULL") != "1",
                    reason="opt-in (GM_TEST_CONFIG4_FULL=1): ~8 min of oracle setup + prove on the host cores; "
                           "run by tools/gpu/config4_full.sh, log in profiles/")
def test_groth16_2p24_squaring_chain_real_setup(gm_ctx, oracle):
    """configs[3]'s own circuit: groth16_test.go:120-156's
    refCircuit with 2^24 - 1 squarings (nc = 2^24 constraints, n = 2^24), a real
    toxic-waste setup by the oracle (setup.go:85-349), a satisfying witness.  The
    GPU proof -- host inputs, device-resident R1CS with the wires staged in the
    solver's one-wire levels, plain and precomputed keys -- equals the oracle's
    byte for byte, and the exponent check accepts it."""
    import gnark_mi355x as gm
    cname = "bn254"
    c = pyref.CURVES[cname]
    t0 = time.time()
    r1, W, a, b, cc = R.squaring_chain_fast((1 << 24) - 1, cname, x=3)
    assert r1.domain_size == 1 << 24 and r1.nc == 1 << 24
    tox = R.encode_vec(cname, [t % c.r for t in TOXIC])
    _log("chain 2^24 built (%.0f s); oracle setup" % (time.time() - t0))
    pk = oracle.g16_setup(cname, r1, tox)
    rb, sb = R.encode_vec(cname, [0x2424242424]), R.encode_vec(cname, [0x4242424242])
    _log("oracle setup done (%.0f s); oracle prove" % (time.time() - t0))
    exp = oracle.g16_prove(cname, pk, r1.nb_public, W, a, b, cc, rb, sb)
    _log("oracle prove done (%.0f s); exponent check" % (time.time() - t0))
    assert oracle.g16_check(cname, r1, tox, W, rb, sb, *exp) == 7
    _log("oracle proof accepted (%.0f s)" % (time.time() - t0))
    hpk = {k: v for k, v in pk.items() if k != "sizes"}
    # the resident system: one term per row and matrix, coefficient id 1 (= one) of
    # gnark's CoeffTable head (0, 1, 2, -1, -2)
    enc = lambda v: (v * (1 << 256) % c.r).to_bytes(32, "little")
    table = b"".join(enc(v) for v in (0, 1, 2, c.r - 1, c.r - 2))
    ones = np.ones(r1.nc, np.uint32)
    h = gm.R1CS(gm_ctx, cname, r1.nc, r1.nb_wires, r1.rowptr, [ones, ones, ones], r1.wires, table)
    try:
        for precompute in (False, True):
            tu = time.time()
            dpk = gm.ProvingKey(gm_ctx, cname, hpk, r1.domain_size, r1.nb_wires, r1.nb_public, precompute=precompute)
            _log("key upload (precompute=%s) %.2f s" % (precompute, time.time() - tu))
            try:
                tp = time.time()
                got = dpk.prove(W, a, b, cc, rb, sb)
                _log("host-input prove %.1f ms" % ((time.time() - tp) * 1e3))
                assert got == exp, precompute
                st = dpk.stage(r1.nc)
                try:
                    ns = st.replay_chain(W, 3, r1.nc)  # one wire per solver level, gathered as the Go hook does
                    got_st = st.prove_r1cs(h, rb, sb)
                finally:
                    st.free()
                _log("staged one-wire levels: %.1f ns per level host side" % ns)
                assert got_st == exp, precompute
            finally:
                dpk.free()
            _log("gpu proofs (precompute=%s) match the oracle" % precompute)
    finally:
        h.free()
    assert oracle.g16_check(cname, r1, tox, W, rb, sb, *got) == 7
