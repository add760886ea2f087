"""End-to-end Groth16 parity: gm_g16_prove (HIP; replaces icicle_bn254.Prove,
backend/groth16/bn254/icicle/icicle.go:133-422) vs the oracle's restatement of
groth16_bn254.Prove (backend/groth16/bn254/prove.go:62-325) on the same pk,
witness and (r, s) -- the proof elements Ar, Bs, Krs must be byte-identical
(SURVEY.md §0.4), and must satisfy the verification equation in the exponent
for the known toxic waste (equivalent of groth16.Verify, verify.go:49-150)."""
import pytest

import pyref
import r1cs as R

pytestmark = pytest.mark.gpu

TOXIC = [0x1D5A2B3C4D5E6F708192A3B4C5D6E7F8091A2B3C4D5E6F708192A3B4C5D6E7,
         0x2E6B3C4D5E6F708192A3B4C5D6E7F8091A2B3C4D5E6F708192A3B4C5D6E7F8,
         0x3F7C4D5E6F708192A3B4C5D6E7F8091A2B3C4D5E6F708192A3B4C5D6E7F809,
         0x0A8D5E6F708192A3B4C5D6E7F8091A2B3C4D5E6F708192A3B4C5D6E7F8091A,
         0x1B9E6F708192A3B4C5D6E7F8091A2B3C4D5E6F708192A3B4C5D6E7F8091A2B]


def _prove_both(gm_ctx, oracle, cname, r1, W, rr, ss, precompute=False):
    import gnark_mi355x as gm
    c = pyref.CURVES[cname]
    tox = R.encode_vec(cname, [t % c.r for t in TOXIC])
    pk = oracle.g16_setup(cname, r1, tox)
    a, b, cc = r1.solve_abc(W)
    enc = lambda v: R.encode_vec(cname, v)
    rb, sb = enc([rr]), enc([ss])
    exp = oracle.g16_prove(cname, pk, r1.nb_public, enc(W), enc(a), enc(b), enc(cc), rb, sb)
    dpk = gm.ProvingKey(gm_ctx, cname, pk, r1.domain_size, r1.nb_wires, r1.nb_public, precompute=precompute)
    try:
        got = dpk.prove(enc(W), enc(a), enc(b), enc(cc), rb, sb)
    finally:
        dpk.free()
    ok = oracle.g16_check(cname, r1, tox, enc(W), rb, sb, *got)
    return exp, got, ok


@pytest.mark.parametrize("cname", ["bn254", "bls12377"])
def test_groth16_cubic(gm_ctx, oracle, cname):
    """examples/cubic (BASELINE config 1 circuit) -- n = 4."""
    r1, W = R.cubic_circuit(cname)
    exp, got, ok = _prove_both(gm_ctx, oracle, cname, r1, W, 0x1234567, 0x7654321)
    assert got == exp
    assert ok == 7


@pytest.mark.parametrize("cname,k", [("bn254", 15), ("bn254", 1023), ("bn254", 4000),
                                     ("bls12377", 511)])
def test_groth16_squaring_chain(gm_ctx, oracle, cname, k):
    """refCircuit of backend/groth16/groth16_test.go:120-156 with k squarings."""
    r1, W = R.squaring_chain(k, cname, x=2)
    exp, got, ok = _prove_both(gm_ctx, oracle, cname, r1, W, 0xABCDEF0123, 0x13579BDF)
    assert got == exp
    assert ok == 7


@pytest.mark.parametrize("cname,k", [("bn254", 15), ("bn254", 4000), ("bls12377", 511)])
def test_groth16_precomputed_pk(gm_ctx, oracle, cname, k):
    """GM_PK_PRECOMPUTE (fixed-base window copies of every pk array): the proof
    is byte-identical to the CPU restatement."""
    r1, W = R.squaring_chain(k, cname, x=3)
    exp, got, ok = _prove_both(gm_ctx, oracle, cname, r1, W, 0x2468ACE, 0x1357BDF, precompute=True)
    assert got == exp
    assert ok == 7


def test_groth16_rejects_bad_witness(gm_ctx, oracle):
    """A proof from an unsatisfying witness must fail the exponent check."""
    r1, W = R.squaring_chain(63, "bn254")
    W = list(W)
    W[10] = (W[10] + 1) % pyref.BN254.r
    exp, got, ok = _prove_both(gm_ctx, oracle, "bn254", r1, W, 5, 7)
    assert got == exp  # same (invalid) computation on both sides
    assert ok != 7


def test_groth16_k_wire_filter(gm_ctx, oracle):
    """BSB22-style K filter (prove.go:243-245): wires removed from the K MSM are
    given by the k_wires index map of the device pk.  Expected: the oracle prover
    on the full pk with the removed wires' K points set to infinity (so they
    contribute nothing)."""
    import numpy as np
    import gnark_mi355x as gm
    cname = "bn254"
    c = pyref.CURVES[cname]
    r1, W = R.squaring_chain(200, cname, x=3)
    tox = R.encode_vec(cname, [t % c.r for t in TOXIC])
    pk = oracle.g16_setup(cname, r1, tox)
    enc = lambda v: R.encode_vec(cname, v)
    a, b, cc = r1.solve_abc(W)
    rb, sb = enc([11]), enc([13])
    nbk = r1.nb_wires - r1.nb_public
    drop = {3, 17, 18, 150}
    keep = [i for i in range(nbk) if i not in drop]
    g1b = gm.point_bytes(cname, False)
    K = np.frombuffer(pk["g1_K"], np.uint8).reshape(nbk, g1b)
    pk_inf = dict(pk)
    Kz = K.copy()
    Kz[sorted(drop)] = 0
    pk_inf["g1_K"] = Kz.reshape(-1)
    exp = oracle.g16_prove(cname, pk_inf, r1.nb_public, enc(W), enc(a), enc(b), enc(cc), rb, sb)
    pk_sub = dict(pk)
    pk_sub["g1_K"] = K[keep].reshape(-1)
    pk_sub["k_wires"] = [r1.nb_public + i for i in keep]
    dpk = gm.ProvingKey(gm_ctx, cname, pk_sub, r1.domain_size, r1.nb_wires, r1.nb_public)
    try:
        got = dpk.prove(enc(W), enc(a), enc(b), enc(cc), rb, sb)
    finally:
        dpk.free()
    assert got == exp


@pytest.mark.parametrize("cname,k,world,precompute", [("bn254", 1023, 2, False), ("bn254", 4000, 3, True),
                                                      ("bls12377", 511, 2, False), ("bn254", 15, 4, False)])
def test_groth16_sharded_partials(gm_ctx, oracle, cname, k, world, precompute):
    """BASELINE config 4 data path on one GPU: every rank's pk shard
    (gm_g16_pk_upload_shard) and partial MSM sums (gm_g16_prove_partial) are
    computed in turn, summed and finished on the host (gm_g16_finish): the proof
    must be byte-identical to the CPU restatement.  world=4 at n=16 leaves
    ragged and tiny shards."""
    import gnark_mi355x as gm
    c = pyref.CURVES[cname]
    r1, W = R.squaring_chain(k, cname, x=5)
    tox = R.encode_vec(cname, [t % c.r for t in TOXIC])
    pk = oracle.g16_setup(cname, r1, tox)
    a, b, cc = r1.solve_abc(W)
    enc = lambda v: R.encode_vec(cname, v)
    rb, sb = enc([0x5151]), enc([0x7373])
    exp = oracle.g16_prove(cname, pk, r1.nb_public, enc(W), enc(a), enc(b), enc(cc), rb, sb)
    n = r1.domain_size
    parts = []
    for rank in range(world):
        dpk = gm.ProvingKey(gm_ctx, cname, pk, n, r1.nb_wires, r1.nb_public, precompute=precompute,
                            shard=(rank, world))
        bufs = []
        try:
            Wd = gm_ctx.copy_to_device(enc(W))
            bufs.append(Wd)
            abc = []
            for v in (a, b, cc):
                d = gm_ctx.malloc(32 * n)
                d.write(bytes(32 * n))
                d.write(enc(v))
                abc.append(d)
            bufs += abc
            parts.append(dpk.prove_partial_device(Wd, *abc, len(a)))
        finally:
            for x in bufs:
                x.free()
            dpk.free()
    got = gm.g16_finish(cname, dpk._h, gm.g16_reduce_partials(cname, parts), rb, sb)
    assert got == exp


@pytest.mark.parametrize("cname,k,ndev", [("bn254", 1023, 2), ("bn254", 15, 5), ("bls12377", 511, 3)])
def test_groth16_multi_contexts_small(gm_ctx, oracle, cname, k, ndev):
    """gm_g16_prove_multi on `ndev` contexts of the one GPU (ragged and tiny
    shards at n = 16 with 5 devices): byte-identical to the CPU restatement and
    accepted by the exponent check."""
    import gnark_mi355x as gm
    c = pyref.CURVES[cname]
    r1, W = R.squaring_chain(k, cname, x=9)
    tox = R.encode_vec(cname, [t % c.r for t in TOXIC])
    pk = oracle.g16_setup(cname, r1, tox)
    a, b, cc = r1.solve_abc(W)
    enc = lambda v: R.encode_vec(cname, v)
    rb, sb = enc([0x1111]), enc([0x2222])
    exp = oracle.g16_prove(cname, pk, r1.nb_public, enc(W), enc(a), enc(b), enc(cc), rb, sb)
    with gm.Multi([0] * ndev) as m:
        mpk = gm.ProvingKeyMulti(m, cname, pk, r1.domain_size, r1.nb_wires, r1.nb_public)
        try:
            got = mpk.prove(enc(W), enc(a), enc(b), enc(cc), rb, sb)
        finally:
            mpk.free()
    assert got == exp
    assert oracle.g16_check(cname, r1, tox, enc(W), rb, sb, *got) == 7


@pytest.mark.parametrize("cname,precompute", [("bn254", False), ("bn254", True), ("bls12377", False)])
def test_groth16_multi_forced_peer_copies(gm_ctx, oracle, monkeypatch, cname, precompute):
    """The peer-copy branches of the multi-device prover -- b / c of computeH
    copied to device 0 (groth16.hip compute_h chains) and the h slices copied to
    the Z-MSM shards (hipMemcpyPeerAsync) -- forced on the one-GPU box with
    GM_MULTI_FORCE_PEER=1 (4 contexts of device 0): the proof is byte-identical
    to the oracle's."""
    import gnark_mi355x as gm
    monkeypatch.setenv("GM_MULTI_FORCE_PEER", "1")
    c = pyref.CURVES[cname]
    r1, W = R.squaring_chain(2000 if cname == "bn254" else 511, cname, x=5)
    tox = R.encode_vec(cname, [t % c.r for t in TOXIC])
    pk = oracle.g16_setup(cname, r1, tox)
    a, b, cc = r1.solve_abc(W)
    enc = lambda v: R.encode_vec(cname, v)
    rb, sb = enc([0x3131]), enc([0x4242])
    exp = oracle.g16_prove(cname, pk, r1.nb_public, enc(W), enc(a), enc(b), enc(cc), rb, sb)
    with gm.Multi([0] * 4) as m:
        mpk = gm.ProvingKeyMulti(m, cname, pk, r1.domain_size, r1.nb_wires, r1.nb_public, precompute=precompute)
        try:
            got = mpk.prove(enc(W), enc(a), enc(b), enc(cc), rb, sb)
            got2 = mpk.prove(enc(W), enc(a), enc(b), enc(cc), rb, sb)
        finally:
            mpk.free()
    assert got == exp and got2 == exp
    assert oracle.g16_check(cname, r1, tox, enc(W), rb, sb, *got) == 7


@pytest.mark.parametrize("cname,ncommit,precompute", [("bn254", 1, False), ("bn254", 2, True),
                                                      ("bls12377", 2, False)])
def test_groth16_bsb22_commitments(gm_ctx, oracle, cname, ncommit, precompute):
    """A circuit with one / two BSB22 commitments (prove.go:82-139) at n = 2^13:
    the oracle solves it through the overridden commitment hint, proves and is
    verified in the exponent; the device side gets the K filter exactly as
    kWires() computes it (integration/go/icicle_bn254/icicle.go; prove.go:243-245)
    and the Pedersen commitments, proofs of knowledge and the fold run as device
    MSMs (gm_msm; pedersen Commit / ProveKnowledge are MultiExps).  Every proof
    element must equal the oracle's byte for byte."""
    import numpy as np
    import gnark_mi355x as gm
    c = pyref.CURVES[cname]
    r1, info, solve = R.commitment_chain(4100, cname, ncommit)
    assert r1.domain_size == 1 << 13
    tox = [t % c.r for t in TOXIC]
    sig = [0x5151515151 + 7 * i for i in range(ncommit)]
    pk = oracle.g16_setup_bsb22(cname, r1, info, tox, sig)
    exp = oracle.g16_prove_bsb22(cname, pk, r1, info, solve, 0x1357, 0x2468)
    assert oracle.bsb22_check(cname, r1, pk, info, exp, sig)
    # K filter of the Go hook (kWires): private wires minus committed and commitment wires
    drop = set(w for ci in info for w in ci["private_committed"]) | set(ci["commitment_index"] for ci in info)
    kw = [w for w in range(r1.nb_public, r1.nb_wires) if w not in drop]
    assert kw == pk["k_wires"]
    dpk = gm.ProvingKey(gm_ctx, cname, dict(pk, k_wires=kw), r1.domain_size, r1.nb_wires, r1.nb_public,
                        precompute=precompute)
    try:
        got = dpk.prove(exp["Wb"], exp["a"], exp["b"], exp["c"], exp["rb"], exp["sb"])
    finally:
        dpk.free()
    assert got == (exp["ar"], exp["bs"], exp["krs"])
    # Pedersen side on the device
    W = exp["W"]
    enc = lambda vals: R.encode_vec(cname, vals)
    g1b = gm.point_bytes(cname, False)
    poks = b""
    for i, ci in enumerate(info):
        vals = enc([W[w] for w in ci["private_committed"]])
        m = len(ci["private_committed"])
        S = gm_ctx.copy_to_device(vals)
        for key, want in (("basis", exp["commitments"][i]), ("basis_sigma", None)):
            P = gm_ctx.copy_to_device(pk["ck"][i][key])
            aff = gm_ctx.msm(cname, S, P, m)[1]
            P.free()
            if want is not None:
                assert aff == want, ("commitment", i)
            else:
                poks += aff
        S.free()
    chal = pyref.pok_challenge(c, [W[ci["commitment_index"]] for ci in info])
    S = gm_ctx.copy_to_device(enc([pow(chal, i, c.r) for i in range(ncommit)]))
    P = gm_ctx.copy_to_device(poks)
    assert gm_ctx.msm(cname, S, P, ncommit)[1] == exp["pok"]
    S.free()
    P.free()
    assert len(poks) == ncommit * g1b


@pytest.mark.parametrize("precompute", [False, True])
@pytest.mark.parametrize("shape", ["chain", "copy"])
def test_groth16_shared_wire_plan_on_off(gm_ctx, oracle, monkeypatch, precompute, shape):
    """The shared wire plan (one digit / sort plan over the wires for the A, B,
    B2 and K MSMs, groth16.hip pk_setup_wire_plan) against per-array plans
    (GM_G16_WIRE_PLAN=0): same proof, equal to the oracle's.  'chain' shares
    A, B and K through wire maps (wires without a point are skipped entries);
    'copy' (w_{j+1} = w_j * ONE: B holds one point) shares A and K only and B /
    B2 keep their own plan."""
    import gnark_mi355x as gm
    cname = "bn254"
    c = pyref.CURVES[cname]
    if shape == "chain":
        r1, W = R.squaring_chain(3000, cname, x=5)
    else:
        k = 3000
        cons = [([(2 + j, 1)], [(0, 1)], [(3 + j, 1)]) for j in range(k)]
        cons.append(([(0, 1)], [(2 + k, 1)], [(1, 1)]))
        r1 = R.R1CS(cname, nb_public=2, nb_wires=3 + k, constraints=cons)
        W = [1, 5] + [5] * (k + 1)
        assert r1.is_satisfied(W)
    tox = R.encode_vec(cname, [t % c.r for t in TOXIC])
    pk = oracle.g16_setup(cname, r1, tox)
    a, b, cc = r1.solve_abc(W)
    enc = lambda v: R.encode_vec(cname, v)
    rb, sb = enc([0xABC]), enc([0xDEF])
    exp = oracle.g16_prove(cname, pk, r1.nb_public, enc(W), enc(a), enc(b), enc(cc), rb, sb)
    for flag in ("1", "0"):
        monkeypatch.setenv("GM_G16_WIRE_PLAN", flag)
        dpk = gm.ProvingKey(gm_ctx, cname, pk, r1.domain_size, r1.nb_wires, r1.nb_public, precompute=precompute)
        try:
            assert dpk.prove(enc(W), enc(a), enc(b), enc(cc), rb, sb) == exp, flag
        finally:
            dpk.free()


@pytest.mark.parametrize("frac,expect", [("0.6", True), ("0.000000001", False)])
def test_groth16_precompute_auto(gm_ctx, oracle, monkeypatch, frac, expect):
    """GM_PK_PRECOMPUTE_AUTO (the Go hook's default): the key takes the window
    copies when they fit GM_PK_PRECOMPUTE_FRAC of the free device memory, else
    stays plain; either way the proof is the oracle's.  The shared wire plan's
    arrays are expanded in gnark layout before the precomputation (no
    compacted precomputed copy), which this key exercises (3 dropped A wires)."""
    import gnark_mi355x as gm
    cname = "bn254"
    c = pyref.CURVES[cname]
    r1, W = R.squaring_chain(2000, cname, x=7)
    tox = R.encode_vec(cname, [t % c.r for t in TOXIC])
    pk = oracle.g16_setup(cname, r1, tox)
    a, b, cc = r1.solve_abc(W)
    enc = lambda v: R.encode_vec(cname, v)
    rb, sb = enc([0x5151]), enc([0x7373])
    exp = oracle.g16_prove(cname, pk, r1.nb_public, enc(W), enc(a), enc(b), enc(cc), rb, sb)
    monkeypatch.setenv("GM_PK_PRECOMPUTE_FRAC", frac)
    dpk = gm.ProvingKey(gm_ctx, cname, pk, r1.domain_size, r1.nb_wires, r1.nb_public, precompute="auto")
    try:
        assert dpk.precomputed is expect
        assert dpk.prove(enc(W), enc(a), enc(b), enc(cc), rb, sb) == exp
    finally:
        dpk.free()


@pytest.mark.parametrize("precompute", [False, True])
def test_groth16_second_msm_stream_with_async_msm_pending(gm_ctx, oracle, monkeypatch, precompute):
    """GM_G16_MSM_STREAMS=1 (the B, B2 and Z MSMs on the prove's own second
    stream): host-input and device-input proofs equal the oracle's, also while a
    gm_msm_async MSM is pending on the same context (its slot stream is not the
    prove's), and that MSM's result is right."""
    import gnark_mi355x as gm
    monkeypatch.setenv("GM_G16_MSM_STREAMS", "1")
    cname = "bn254"
    c = pyref.CURVES[cname]
    r1, W = R.squaring_chain(3000, cname, x=6)
    tox = R.encode_vec(cname, [t % c.r for t in TOXIC])
    pk = oracle.g16_setup(cname, r1, tox)
    a, b, cc = r1.solve_abc(W)
    enc = lambda v: R.encode_vec(cname, v)
    rb, sb = enc([0x7171]), enc([0x8282])
    exp = oracle.g16_prove(cname, pk, r1.nb_public, enc(W), enc(a), enc(b), enc(cc), rb, sb)
    n = 1 << 16
    S = gm_ctx.random_scalars(cname, n, seed=0x91)
    K = gm_ctx.random_scalars(cname, n, seed=0x92)
    P = gm_ctx.batch_mul_base(cname, False, gm.generator(cname), K, n)
    msm_exp = oracle.msm(cname, False, S.to_host(), P.to_host())
    dpk = gm.ProvingKey(gm_ctx, cname, pk, r1.domain_size, r1.nb_wires, r1.nb_public, precompute=precompute)
    try:
        assert dpk.prove(enc(W), enc(a), enc(b), enc(cc), rb, sb) == exp
        pend = gm_ctx.msm_async(cname, S, P, n)
        got = dpk.prove(enc(W), enc(a), enc(b), enc(cc), rb, sb)
        assert pend.wait()[1] == msm_exp
        assert got == exp
    finally:
        dpk.free()
        for x in (S, K, P):
            x.free()


def test_gm_trim_releases_and_recreates(gm_ctx, oracle):
    """gm_trim frees what the context keeps between calls (arenas, the host-input
    a / b / c buffer, the pinned ring, NTT tables); later calls re-create them and
    give the same results.  Refused while an async MSM is pending."""
    import gnark_mi355x as gm
    cname = "bn254"
    c = pyref.CURVES[cname]
    r1, W = R.squaring_chain(1500, cname, x=4)
    tox = R.encode_vec(cname, [t % c.r for t in TOXIC])
    pk = oracle.g16_setup(cname, r1, tox)
    a, b, cc = r1.solve_abc(W)
    enc = lambda v: R.encode_vec(cname, v)
    rb, sb = enc([0x1a1a]), enc([0x2b2b])
    exp = oracle.g16_prove(cname, pk, r1.nb_public, enc(W), enc(a), enc(b), enc(cc), rb, sb)
    dpk = gm.ProvingKey(gm_ctx, cname, pk, r1.domain_size, r1.nb_wires, r1.nb_public)
    S = gm_ctx.random_scalars(cname, 5000, seed=0x31)
    K = gm_ctx.random_scalars(cname, 5000, seed=0x32)
    P = gm_ctx.batch_mul_base(cname, False, gm.generator(cname), K, 5000)
    try:
        assert dpk.prove(enc(W), enc(a), enc(b), enc(cc), rb, sb) == exp
        gm_ctx.trim()
        assert dpk.prove(enc(W), enc(a), enc(b), enc(cc), rb, sb) == exp
        pend = gm_ctx.msm_async(cname, S, P, 5000)
        with pytest.raises(gm.GmError, match="pending"):
            gm_ctx.trim()
        assert pend.wait()[1] == oracle.msm(cname, False, S.to_host(), P.to_host())
        gm_ctx.trim()
        assert gm_ctx.msm(cname, S, P, 5000)[1] == oracle.msm(cname, False, S.to_host(), P.to_host())
    finally:
        dpk.free()
        for x in (S, K, P):
            x.free()
