"""CPU tests of the oracle (no GPU): pins the restatements against the values
the reference itself holds, then checks the C++ restatement against the
pure-Python one and against the committed golden fixtures."""
import glob
import json
import os

import pytest

import pyref
import r1cs as R

HERE = os.path.dirname(os.path.abspath(__file__))
GOLDEN = os.path.join(HERE, "golden")


def _load(name):
    with open(os.path.join(GOLDEN, name + ".json")) as f:
        return json.load(f)


# ---- reference-pinned constants ------------------------------------------------

def test_bn254_twist_vectors_from_reference():
    """std/algebra/emulated/sw_bn254/pairing_test.go:333-345 (point NOT on the twist)
    and :394-404 (point on the curve but NOT in G2)."""
    c = pyref.BN254
    G2 = pyref.Group(c, True)
    not_on = ((0x119606e6d3ea97cea4eff54433f5c7dbc026b8d0670ddfbe6441e31225028d31,
               0x1d3df5be6084324da6333a6ad1367091ca9fbceb70179ec484543a58b8cb5d63),
              (0x1b9a36ea373fe2c5b713557042ce6deb2907d34e12be595f9bbe84c144de86ef,
               0x49fe60975e8c78b7b31a6ed16a338ac8b28cf6a065cfd2ca47e9402882518ba0 % c.p))
    assert not G2.on_curve(not_on)
    on_not_sub = ((0x07192b9fd0e2a32e3e1caa8e59462b757326d48f641924e6a1d00d66478913eb,
                   0x15ce93f1b1c4946dd6cfbb3d287d9c9a1cdedb264bda7aada0844416d8a47a63),
                  (0x0fa65a9b48ba018361ed081e3b9e958451de5d9e8ae0bd251833ebb4b2fafc96,
                   0x06e1f5e20f68f6dfa8a91a3bea048df66d9eaf56cc7f11215401f7e05027e0c6))
    assert G2.on_curve(on_not_sub)
    assert G2.mul(on_not_sub, c.r) is not None  # not in the r-torsion subgroup


@pytest.mark.parametrize("cname", ["bn254", "bls12377"])
def test_curve_constants(cname):
    c = pyref.CURVES[cname]
    for g2 in (False, True):
        G = pyref.Group(c, g2)
        assert G.on_curve(G.generator())
        assert G.mul(G.generator(), c.r) is None
    # 2-adic root of unity of exact order 2^s, = g^((r-1)/2^s)
    w = c.omega_max
    assert pow(w, 1 << c.two_adicity, c.r) == 1
    assert pow(w, 1 << (c.two_adicity - 1), c.r) != 1
    assert pow(c.coset_gen, (c.r - 1) >> c.two_adicity, c.r) == w


def test_bn254_double_generator_kat():
    """2*G1 for BN254 (SURVEY.md §8c known answer)."""
    G = pyref.Group(pyref.BN254, False)
    P = G.mul(G.generator(), 2)
    assert P == (0x030644e72e131a029b85045b68181585d97816a916871ca8d3c208c16d87cfd3,
                 0x15ed738c0e0a7c92e7845f96b2ae9c0a68a6a449e3538fc7ff3ebf7a5a18a2c4)


def test_filter_heap_reference_vectors():
    """backend/groth16/bn254/utils_test.go:17-38."""
    e = [0, 1, 2, 3]
    assert pyref.filter_heap(e, 0, [1, 2]) == [0, 3]
    assert pyref.filter_heap(e[1:], 1, [1, 2]) == [3]
    assert pyref.filter_heap(e, 0, [1, 1, 2]) == [0, 3]
    assert pyref.filter_heap(e[1:], 1, [1, 1, 2]) == [3]


def test_bitreverse_matches_setup():
    """setup.go:690-700 bitReverse."""
    assert pyref.bit_reverse(list(range(8))) == [0, 4, 2, 6, 1, 5, 3, 7]


# ---- C++ restatement vs golden fixtures (pure-Python restatement outputs) ------

@pytest.mark.parametrize("name", sorted(os.path.basename(p)[:-5] for p in glob.glob(os.path.join(GOLDEN, "msm_*.json"))))
def test_oracle_msm_golden(oracle, name):
    g = _load(name)
    got = oracle.msm(g["curve"], g["g2"], bytes.fromhex(g["scalars"]), bytes.fromhex(g["points"]))
    assert got.hex() == g["expected_affine"]
    got = oracle.msm(g["curve"], g["g2"], bytes.fromhex(g["scalars"]), bytes.fromhex(g["points"]), naive=True)
    assert got.hex() == g["expected_affine"]


@pytest.mark.parametrize("cname", ["bn254", "bls12377"])
def test_oracle_ntt_golden(oracle, cname):
    g = _load("ntt_" + cname)
    x = bytes.fromhex(g["input"])
    for mode, exp in g["outputs"].items():
        inverse, dit, coset = (int(ch) for ch in mode)
        assert oracle.fft(cname, x, inverse, dit, coset).hex() == exp, mode


@pytest.mark.parametrize("name", ["h_cubic_bn254", "h_cubic_bls12377", "h_squaring15_bn254",
                                  "h_squaring15_bls12377"])
def test_oracle_compute_h_golden(oracle, name):
    g = _load(name)
    got = oracle.compute_h(g["curve"], bytes.fromhex(g["a"]), bytes.fromhex(g["b"]), bytes.fromhex(g["c"]), g["n"])
    assert got.hex() == g["h_bitrev"]


def _pk_from_fixture(g):
    import numpy as np
    pk = {k: np.frombuffer(bytes.fromhex(v), np.uint8).copy() for k, v in g["pk"].items()}
    fpb = 32 if g["curve"] == "bn254" else 48
    nbK = g["nb_wires"] - g["nb_public"]
    pk["sizes"] = np.array([g["n"], g["nb_wires"], len(pk["g1_A"]) // (2 * fpb), len(pk["g1_B"]) // (2 * fpb), nbK],
                           dtype=np.uint64)
    return pk


@pytest.mark.parametrize("cname", ["bn254", "bls12377"])
def test_oracle_groth16_golden(oracle, cname):
    g = _load("groth16_cubic_" + cname)
    pk = _pk_from_fixture(g)
    h = lambda k: bytes.fromhex(g[k])
    ar, bs, krs = oracle.g16_prove(cname, pk, g["nb_public"], h("wires"), h("a"), h("b"), h("c"), h("r"), h("s"))
    assert (ar.hex(), bs.hex(), krs.hex()) == (g["expected"]["Ar"], g["expected"]["Bs"], g["expected"]["Krs"])
    r1, W = R.cubic_circuit(cname)
    assert oracle.g16_check(cname, r1, h("toxic"), h("wires"), h("r"), h("s"), ar, bs, krs) == 7


@pytest.mark.parametrize("cname", ["bn254", "bls12377"])
def test_oracle_setup_matches_pyref(oracle, cname):
    """The C++ Setup restatement reproduces the pure-Python one (fixture pk)."""
    g = _load("groth16_cubic_" + cname)
    r1, W = R.cubic_circuit(cname)
    pk = oracle.g16_setup(cname, r1, bytes.fromhex(g["toxic"]))
    for k, v in g["pk"].items():
        assert pk[k].tobytes().hex() == v, k


# ---- C++ restatement vs pyref at random sizes -------------------------------------

@pytest.mark.parametrize("cname", ["bn254", "bls12377"])
def test_oracle_pippenger_vs_naive(oracle, cname):
    c = pyref.CURVES[cname]
    n = 300
    sc = pyref.random_scalars(c, n, 5)
    ks = R.encode_vec(cname, pyref.random_scalars(c, n, 6))
    pts = oracle.batch_mul_base(cname, False, oracle.generator(cname, False), ks)
    sb = R.encode_vec(cname, sc)
    assert oracle.msm(cname, False, sb, pts) == oracle.msm(cname, False, sb, pts, naive=True)


@pytest.mark.parametrize("cname", ["bn254", "bls12377"])
def test_oracle_groth16_random_circuit(oracle, cname):
    r1, W = R.squaring_chain(200, cname, x=7)
    tox = R.encode_vec(cname, [11, 22, 33, 44, 55])
    pk = oracle.g16_setup(cname, r1, tox)
    a, b, cc = r1.solve_abc(W)
    enc = lambda v: R.encode_vec(cname, v)
    rb, sb = enc([3]), enc([4])
    proof = oracle.g16_prove(cname, pk, r1.nb_public, enc(W), enc(a), enc(b), enc(cc), rb, sb)
    assert oracle.g16_check(cname, r1, tox, enc(W), rb, sb, *proof) == 7


# ---- BSB22 commitments (prove.go:82-139) --------------------------------------

def test_expand_message_xmd_rfc9380_vectors():
    """RFC 9380 appendix K.1 (expand_message_xmd, SHA-256,
    DST "QUUX-V01-CS02-with-expander-SHA256-128"): the published algorithm
    gnark-crypto's fr.Hash / hash_to_field.New build on."""
    dst = b"QUUX-V01-CS02-with-expander-SHA256-128"
    assert pyref.expand_message_xmd(b"", dst, 0x20).hex() == \
        "68a985b87eb6b46952128911f2a4412bbc302a9d759667f87f7a21d803f07235"
    assert pyref.expand_message_xmd(b"abc", dst, 0x20).hex() == \
        "d8ccab23b5985ccea865c6c97b6e5b8350e794e603b4b97902f53a8a0d605615"
    assert pyref.expand_message_xmd(b"", dst, 0x80).hex().startswith(
        "af84c27ccfd45d41914fdff5df25293e221afc53d8ad2ac06d5e3e29485dadbe")


def test_bsb22_serialization_shapes():
    """SerializeCommitment (constraint/commitment.go:70-82) = Marshal(D) (the
    uncompressed point, verify.go:88) || each committed public value as
    (fr.Bits-1)/8+1 big-endian bytes; fr.Hash takes 16 + 32 = 48 bytes per element."""
    for cname in ("bn254", "bls12377"):
        c = pyref.CURVES[cname]
        G = pyref.Group(c, False)
        D = G.mul(G.generator(), 12345)
        s = pyref.serialize_commitment(pyref.marshal_g1(c, D), [7, c.r - 1], pyref.fr_byte_len(c))
        assert len(s) == 2 * 8 * c.fp_limbs + 2 * 32
        assert s[-32:] == (c.r - 1).to_bytes(32, "big")
        assert pyref.marshal_g1(c, D)[:8 * c.fp_limbs] == D[0].to_bytes(8 * c.fp_limbs, "big")
        v = pyref.hash_to_fr(c, b"msg", pyref.COMMITMENT_DST, 2)
        assert len(v) == 2 and all(0 <= x < c.r for x in v) and v[0] != v[1]


@pytest.mark.parametrize("cname,ncommit", [("bn254", 1), ("bn254", 2), ("bls12377", 2)])
def test_oracle_groth16_bsb22_verifies(oracle, cname, ncommit):
    """The oracle's prover with BSB22 commitments (hint override, Pedersen
    commit / proof of knowledge, fold, K filter) produces proofs that satisfy
    verify.go's equation (exponent form, with the commitment wires and the
    private committed wires on the verifier's side) and the folded PoK
    statement; a wrong PoK or a missing K filter is rejected."""
    r1, info, solve = R.commitment_chain(40, cname, ncommit)
    tox = [0x1234567 + i * 0x99999 for i in range(5)]
    sig = [0xABCDEF + 17 * i for i in range(ncommit)]
    pk = oracle.g16_setup_bsb22(cname, r1, info, tox, sig)
    pr = oracle.g16_prove_bsb22(cname, pk, r1, info, solve, 0x1111, 0x2222)
    assert oracle.bsb22_check(cname, r1, pk, info, pr, sig)
    c = pyref.CURVES[cname]
    bad = dict(pr)
    bad["pok"] = pyref.encode_point(c, pyref.Group(c, False).generator(), False)
    assert not oracle.bsb22_check(cname, r1, pk, info, bad, sig)
    # the same witness proved WITHOUT the K filter double-counts the committed wires
    full = dict(pk)
    full["g1_K"] = pk["g1_K_full"]
    full["sizes"] = pk["sizes"].copy()
    full["sizes"][4] = r1.nb_wires - r1.nb_public
    ar, bs, krs = oracle.g16_prove(cname, full, r1.nb_public, pr["Wb"], pr["a"], pr["b"], pr["c"], pr["rb"], pr["sb"])
    nf = dict(pr, ar=ar, bs=bs, krs=krs)
    assert not oracle.bsb22_check(cname, r1, pk, info, nf, sig)


@pytest.mark.parametrize("cname,g2", [("bn254", False), ("bn254", True), ("bls12377", False), ("bls12377", True)])
def test_oracle_signed_pippenger_vs_unsigned(oracle, cname, g2):
    """The default oracle MSM (signed digits, XYZZ buckets: gnark-crypto
    MultiExp's shape; the bench's CPU baseline) against the unsigned-digit
    Jacobian Pippenger (naive=2), edge scalars included."""
    c = pyref.CURVES[cname]
    for n in (1, 7, 300, 2049):
        sc = pyref.random_scalars(c, n, n + 11)
        sc[0] = c.r - 1
        if n > 3:
            sc[1], sc[2] = 0, 1
        sb = R.encode_vec(cname, sc)
        pts = oracle.batch_mul_base(cname, g2, oracle.generator(cname, g2),
                                    R.encode_vec(cname, pyref.random_scalars(c, n, n + 12)))
        assert oracle.msm(cname, g2, sb, pts) == oracle.msm(cname, g2, sb, pts, naive=2), n


def _glv_module():
    import importlib.util
    spec = importlib.util.spec_from_file_location(
        "glv_constants", os.path.join(HERE, "..", "tools", "glv_constants.py"))
    m = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(m)
    return m


def _hpp_array(name, struct):
    """The uint32 array literal of `name` inside `struct` in csrc/msm_impl.hpp."""
    import re
    src = open(os.path.join(HERE, "..", "gnark-icicle_amd", "csrc", "msm_impl.hpp")).read()
    body = src[src.index("struct %s {" % struct):]
    body = body[:body.index("\n};")]
    fn = body[body.index(name + "(int i)"):]
    lit = fn[fn.index("{", fn.index("a[")) + 1:fn.index("};")]
    return [int(x.rstrip("u"), 16) for x in re.findall(r"0x[0-9a-fA-F]+u", lit)]


def test_bn254_glv_constants_pinned_by_reference():
    """The BN254 GLV endomorphism of the MSM (csrc/msm_impl.hpp GlvBn254) is the
    conjugate of the one the reference holds: std/algebra/emulated/sw_emulated/
    params.go:54-55 (GetBN254Params: Eigenvalue lambda_ref, ThirdRootOne
    omega_ref).  Ours: lambda = r - 1 - lambda_ref = lambda_ref^2 mod r and
    beta = p - 1 - omega_ref = omega_ref^2 mod p; both pairs satisfy
    phi(x, y) = (beta x, y) = [lambda](x, y) on G1, and the device's radix-2^29
    Montgomery beta (and beta^2 for the G2 twist) encode exactly these."""
    c = pyref.BN254
    p, r = c.p, c.r
    lam_ref = 4407920970296243842393367215006156084916469457145843978461
    omega_ref = 2203960485148121921418603742825762020974279258880205651966
    d = _glv_module().derive()
    assert d["lam"] == r - 1 - lam_ref == lam_ref * lam_ref % r
    assert d["beta"] == p - 1 - omega_ref == omega_ref * omega_ref % p
    G = pyref.Group(c, False)
    P = G.mul(G.generator(), 0x1234567)
    assert G.mul(P, lam_ref) == (omega_ref * P[0] % p, P[1])      # the reference's pair
    assert G.mul(P, d["lam"]) == (d["beta"] * P[0] % p, P[1])      # the device's (conjugate) pair

    def r29(x):
        v = x * (1 << 261) % p
        return [(v >> (29 * i)) & ((1 << 29) - 1) for i in range(9)]
    assert _hpp_array("beta29", "GlvBn254") == r29(d["beta"])
    assert _hpp_array("beta29_g2", "GlvBn254") == r29(d["beta"] * d["beta"] % p)
    # the lattice basis the device splits with: a + b lambda = 0 mod r
    assert (d["a1"] + d["b1"] * d["lam"]) % r == 0 and (d["a2"] + d["b2"] * d["lam"]) % r == 0


def _hpp_u64(name, struct):
    """The `static constexpr uint64_t` constants `name` of `struct` (msm_impl.hpp)."""
    import re
    src = open(os.path.join(HERE, "..", "gnark-icicle_amd", "csrc", "msm_impl.hpp")).read()
    body = src[src.index("struct %s {" % struct):]
    body = body[:body.index("\n};")]
    return int(re.search(r"\b%s = (0x[0-9a-fA-F]+)ull" % name, body).group(1), 16)


def _hpp_u64_array(name, struct):
    import re
    src = open(os.path.join(HERE, "..", "gnark-icicle_amd", "csrc", "msm_impl.hpp")).read()
    body = src[src.index("struct %s {" % struct):]
    body = body[:body.index("\n};")]
    fn = body[body.index(name + "(int i)"):]
    lit = fn[fn.index("{", fn.index("a[")) + 1:fn.index("};")]
    return [int(x[:-3], 16) for x in re.findall(r"0x[0-9a-fA-F]+ull", lit)]


def test_bls12377_glv_constants_pinned_by_reference():
    """The BLS12-377 GLV endomorphism of the MSM (csrc/msm_impl.hpp GlvBls377)
    is exactly the one the reference holds in std/algebra/native/sw_bls12377/
    inner.go:58-63: lambda = bls12377lambda, and phi1 (inner.go:26-30, G1)
    multiplies x by thirdRootOne1 while phi2 (:38-42, the G2 twist) multiplies
    by thirdRootOne2 = thirdRootOne1^2 (inner.go:63).  The device's lambda
    (LAM_HI:LAM_LO), its split constant g = floor(2^384 / lambda), and its
    radix-2^29 Montgomery beta / beta^2 (R = 2^406) encode exactly these, and
    [lambda] P = (thirdRootOne1 x, y) holds on G1 and G2 points."""
    c = pyref.CURVES["bls12377"]
    p, r = c.p, c.r
    lam_ref = int.from_bytes(bytes([0x45, 0x22, 0x17, 0xcc, 0x90, 0x00, 0x00, 0x01, 0x0a, 0x11, 0x80, 0x00,
                                    0x00, 0x00, 0x00, 0x00]), "big")
    t1_ref = int.from_bytes(bytes([
        0x09, 0xb3, 0xaf, 0x05, 0xdd, 0x14, 0xf6, 0xec, 0x61, 0x9a, 0xaf, 0x7d, 0x34, 0x59,
        0x4a, 0xab, 0xc5, 0xed, 0x13, 0x47, 0x97, 0x0d, 0xec, 0x00, 0x45, 0x22, 0x17, 0xcc,
        0x90, 0x00, 0x00, 0x00, 0x85, 0x08, 0xc0, 0x00, 0x00, 0x00, 0x00, 0x01]), "big")
    t2_ref = t1_ref * t1_ref % p
    lam_dev = (_hpp_u64("LAM_HI", "GlvBls377") << 64) | _hpp_u64("LAM_LO", "GlvBls377")
    assert lam_dev == lam_ref
    g = _hpp_u64_array("g", "GlvBls377")
    assert sum(v << (64 * i) for i, v in enumerate(g)) == (1 << 384) // lam_ref

    def r29(x):
        v = x * (1 << (29 * 14)) % p
        return [(v >> (29 * i)) & ((1 << 29) - 1) for i in range(14)]
    assert _hpp_array("beta29", "GlvBls377") == r29(t1_ref)
    assert _hpp_array("beta29_g2", "GlvBls377") == r29(t2_ref)
    # the reference's pair is an endomorphism of both groups
    G1, G2 = pyref.Group(c, False), pyref.Group(c, True)
    P = G1.mul(G1.generator(), 0x7654321)
    assert G1.mul(P, lam_ref) == (t1_ref * P[0] % p, P[1])
    Q = G2.mul(G2.generator(), 0x1234)
    LQ = G2.mul(Q, lam_ref)
    assert LQ == ((Q[0][0] * t2_ref % p, Q[0][1] * t2_ref % p), Q[1])
    # and the derivation tool agrees
    d = _glv_module().derive_bls12377()
    assert (d["lam"], d["beta"], d["beta_g2"]) == (lam_ref, t1_ref, t2_ref)
    assert (lam_ref * lam_ref + lam_ref + 1) % r == 0
