"""TEST ORACLE ONLY -- pure-Python big-integer restatement of the MSM / NTT /
computeH arithmetic that gnark's Groth16 prover delegates to gnark-crypto
(CPU) or ICICLE (GPU).  Used only by tests/, the golden-fixture generator and
as a cross-check of the C restatement (oracle/gm_oracle.c).  Never imported by
the product path.

What it restates (reference call sites; the algorithms live in gnark-crypto
v0.14.1-0.20241010154951-6638408a49f3, go.mod:9, which is not vendored):

  * G1Jac.MultiExp / G2Jac.MultiExp        backend/groth16/bn254/prove.go:204,217,237,247,293
    -> msm(): sum_i int(s_i) * P_i, s_i given as Montgomery fr.Element,
       P_i affine with (0,0) = infinity (gnark convention).
  * fft.Domain.FFT / FFTInverse             backend/groth16/bn254/prove.go:372-378,396
    -> fft()/fft_inverse(): DIF = natural in -> bit-reversed out,
       DIT = bit-reversed in -> natural out; OnCoset uses FrMultiplicativeGen.
  * computeH                                backend/groth16/bn254/prove.go:356-399
  * setup Z bit reversal                    backend/groth16/bn254/setup.go:265-267, 690-700
  * filterHeap                              backend/groth16/bn254/prove.go:331-354

Parity status: the reference tree holds NO known-answer vectors for MSM, NTT or
H, so parity against gnark-crypto itself is UNPINNED.  What is
pinned: the curve constants (generators, 2*G1 known answer, 2-adic root
orders, twist coefficients) and the on-curve / subgroup verdicts of the G2
points hard-coded in the reference at
std/algebra/emulated/sw_bn254/pairing_test.go:333-400 (see tests/test_oracle.py).
"""
from __future__ import annotations

import random
from dataclasses import dataclass

# ----------------------------------------------------------------------------
# curve parameters
# ----------------------------------------------------------------------------


@dataclass(frozen=True)
class CurveParams:
    name: str
    p: int
    r: int
    fp_limbs: int          # 64-bit limbs of an fp.Element
    fr_limbs: int          # 64-bit limbs of an fr.Element
    b: int                 # G1: y^2 = x^3 + b
    beta: int              # Fp2 = Fp[u]/(u^2 - beta)
    b2: tuple              # G2 twist coefficient (A0, A1)
    g1: tuple
    g2: tuple              # ((x0, x1), (y0, y1)) or None
    coset_gen: int         # fft FrMultiplicativeGen
    omega_max: int         # generator of the largest 2-adic subgroup of Fr
    two_adicity: int


_BN_P = 21888242871839275222246405745257275088696311157297823662689037894645226208583
_BN_R = 21888242871839275222246405745257275088548364400416034343698204186575808495617


def _bn_b2():
    # 3 / (9 + u) in Fp2 with u^2 = -1
    p = _BN_P
    a0, a1 = 9, 1
    norm = (a0 * a0 + a1 * a1) % p
    inv = pow(norm, -1, p)
    return (3 * a0 * inv % p, (-3 * a1 * inv) % p)


BN254 = CurveParams(
    name="bn254",
    p=_BN_P,
    r=_BN_R,
    fp_limbs=4,
    fr_limbs=4,
    b=3,
    beta=_BN_P - 1,
    b2=_bn_b2(),
    g1=(1, 2),
    g2=((10857046999023057135944570762232829481370756359578518086990519993285655852781,
         11559732032986387107991004021392285783925812861821192530917403151452391805634),
        (8495653923123431417604973247489272438418190587263600148770280649306958101930,
         4082367875863433681332203403145435568316851327593401208105741076214120093531)),
    coset_gen=5,
    omega_max=19103219067921713944291392827692070036145651957329286315305642004821462161904,
    two_adicity=28,
)

_BLS_P = 258664426012969094010652733694893533536393512754914660539884262666720468348340822774968888139573360124440321458177
_BLS_R = 8444461749428370424248824938781546531375899335154063827935233455917409239041

BLS12_377 = CurveParams(
    name="bls12377",
    p=_BLS_P,
    r=_BLS_R,
    fp_limbs=6,
    fr_limbs=4,
    b=1,
    beta=_BLS_P - 5,
    b2=(0, (-pow(5, -1, _BLS_P)) % _BLS_P),   # 1/u with u^2 = -5
    g1=(0x008848defe740a67c8fc6225bf87ff5485951e2caa9d41bb188282c8bd37cb5cd5481512ffcd394eeab9b16eb21be9ef,
        0x01914a69c5102eff1f674f5d30afeec4bd7fb348ca3e52d96d182ad44fb82305c2fe3d3634a9591afd82de55559c8ea6),
    g2=((233578398248691099356572568220835526895379068987715365179118596935057653620464273615301663571204657964920925606294,
         140913150380207355837477652521042157274541796891053068589147167627541651775299824604154852141315666357241556069118),
        (63160294768292073209381361943935198908131692476676907196754037919244929611450776219210369229519898517858833747423,
         149157405641012693445398062341192467754805999074082136895788947234480009303640899064710353187729182149407503257491)),
    coset_gen=22,
    omega_max=8065159656716812877374967518403273466521432693661810619979959746626482506078,
    two_adicity=47,
)

CURVES = {"bn254": BN254, "bls12377": BLS12_377}

# ----------------------------------------------------------------------------
# Fp2 helpers (tuples)
# ----------------------------------------------------------------------------


class F2:
    def __init__(self, c: CurveParams):
        self.p = c.p
        self.beta = c.beta

    def add(self, a, b):
        p = self.p
        return ((a[0] + b[0]) % p, (a[1] + b[1]) % p)

    def sub(self, a, b):
        p = self.p
        return ((a[0] - b[0]) % p, (a[1] - b[1]) % p)

    def neg(self, a):
        p = self.p
        return ((-a[0]) % p, (-a[1]) % p)

    def mul(self, a, b):
        p = self.p
        return ((a[0] * b[0] + self.beta * a[1] * b[1]) % p, (a[0] * b[1] + a[1] * b[0]) % p)

    def inv(self, a):
        p = self.p
        norm = (a[0] * a[0] - self.beta * a[1] * a[1]) % p
        ni = pow(norm, -1, p)
        return (a[0] * ni % p, (-a[1]) * ni % p)

    def is_zero(self, a):
        return a[0] % self.p == 0 and a[1] % self.p == 0


class F1:
    def __init__(self, c: CurveParams):
        self.p = c.p

    def add(self, a, b):
        return (a + b) % self.p

    def sub(self, a, b):
        return (a - b) % self.p

    def neg(self, a):
        return (-a) % self.p

    def mul(self, a, b):
        return a * b % self.p

    def inv(self, a):
        return pow(a, -1, self.p)

    def is_zero(self, a):
        return a % self.p == 0


# ----------------------------------------------------------------------------
# short-Weierstrass group law (a = 0), Jacobian coordinates; None = infinity
# ----------------------------------------------------------------------------


class Group:
    def __init__(self, c: CurveParams, g2: bool):
        self.c = c
        self.F = F2(c) if g2 else F1(c)
        self.b = c.b2 if g2 else c.b % c.p
        self.g2 = g2
        self.zero = (0, 0) if g2 else 0
        self.one = (1, 0) if g2 else 1

    # affine helpers --------------------------------------------------------
    def on_curve(self, P):
        if P is None:
            return True
        F = self.F
        x, y = P
        return F.is_zero(F.sub(F.mul(y, y), F.add(F.mul(F.mul(x, x), x), self.b)))

    def neg(self, P):
        if P is None:
            return None
        return (P[0], self.F.neg(P[1]))

    def to_jac(self, P):
        if P is None:
            return (self.one, self.one, self.zero)
        return (P[0], P[1], self.one)

    def to_aff(self, J):
        F = self.F
        X, Y, Z = J
        if F.is_zero(Z):
            return None
        zi = F.inv(Z)
        zi2 = F.mul(zi, zi)
        return (F.mul(X, zi2), F.mul(Y, F.mul(zi2, zi)))

    def jdbl(self, J):
        F = self.F
        X, Y, Z = J
        if F.is_zero(Z):
            return J
        A = F.mul(X, X)
        B = F.mul(Y, Y)
        C = F.mul(B, B)
        t = F.add(X, B)
        D = F.sub(F.sub(F.mul(t, t), A), C)
        D = F.add(D, D)
        E = F.add(F.add(A, A), A)
        Fv = F.mul(E, E)
        X3 = F.sub(Fv, F.add(D, D))
        C8 = F.add(C, C)
        C8 = F.add(C8, C8)
        C8 = F.add(C8, C8)
        Y3 = F.sub(F.mul(E, F.sub(D, X3)), C8)
        YZ = F.mul(Y, Z)
        Z3 = F.add(YZ, YZ)
        return (X3, Y3, Z3)

    def jadd(self, J1, J2):
        F = self.F
        X1, Y1, Z1 = J1
        X2, Y2, Z2 = J2
        if F.is_zero(Z1):
            return J2
        if F.is_zero(Z2):
            return J1
        Z1Z1 = F.mul(Z1, Z1)
        Z2Z2 = F.mul(Z2, Z2)
        U1 = F.mul(X1, Z2Z2)
        U2 = F.mul(X2, Z1Z1)
        S1 = F.mul(Y1, F.mul(Z2, Z2Z2))
        S2 = F.mul(Y2, F.mul(Z1, Z1Z1))
        if F.is_zero(F.sub(U1, U2)):
            if F.is_zero(F.sub(S1, S2)):
                return self.jdbl(J1)
            return (self.one, self.one, self.zero)
        H = F.sub(U2, U1)
        I = F.add(H, H)
        I = F.mul(I, I)
        Jv = F.mul(H, I)
        rr = F.sub(S2, S1)
        rr = F.add(rr, rr)
        V = F.mul(U1, I)
        X3 = F.sub(F.sub(F.mul(rr, rr), Jv), F.add(V, V))
        S1J = F.mul(S1, Jv)
        Y3 = F.sub(F.mul(rr, F.sub(V, X3)), F.add(S1J, S1J))
        t = F.add(Z1, Z2)
        Z3 = F.mul(F.sub(F.sub(F.mul(t, t), Z1Z1), Z2Z2), H)
        return (X3, Y3, Z3)

    def add(self, P, Q):
        return self.to_aff(self.jadd(self.to_jac(P), self.to_jac(Q)))

    def mul(self, P, k: int):
        """[k]P for a non-negative integer k (double-and-add)."""
        R = self.to_jac(None)
        Jp = self.to_jac(P)
        for bit in bin(k)[2:] if k > 0 else "":
            R = self.jdbl(R)
            if bit == "1":
                R = self.jadd(R, Jp)
        return self.to_aff(R)

    def generator(self):
        c = self.c
        return c.g2 if self.g2 else c.g1

    def msm(self, scalars, points):
        """sum_i scalars[i] * points[i]; scalars are canonical integers mod r.
        Bucket method with 8-bit windows (exact group arithmetic; the result is
        independent of the algorithm)."""
        c = 8
        nbits = self.c.r.bit_length()
        nwin = (nbits + c - 1) // c
        acc = self.to_jac(None)
        for w in reversed(range(nwin)):
            for _ in range(c):
                acc = self.jdbl(acc)
            buckets = [self.to_jac(None) for _ in range(1 << c)]
            for s, P in zip(scalars, points):
                if P is None:
                    continue
                d = (s >> (c * w)) & ((1 << c) - 1)
                if d:
                    buckets[d] = self.jadd(buckets[d], self.to_jac(P))
            run = self.to_jac(None)
            tot = self.to_jac(None)
            for d in range((1 << c) - 1, 0, -1):
                run = self.jadd(run, buckets[d])
                tot = self.jadd(tot, run)
            acc = self.jadd(acc, tot)
        return self.to_aff(acc)


# ----------------------------------------------------------------------------
# gnark memory layout (little-endian 64-bit limbs, Montgomery form)
# ----------------------------------------------------------------------------


def mont_encode(x: int, modulus: int, limbs: int) -> bytes:
    R = 1 << (64 * limbs)
    return (x * R % modulus).to_bytes(8 * limbs, "little")


def mont_decode(b: bytes, modulus: int, limbs: int) -> int:
    R = 1 << (64 * limbs)
    return int.from_bytes(b[: 8 * limbs], "little") * pow(R, -1, modulus) % modulus


def encode_fr(c: CurveParams, x: int) -> bytes:
    return mont_encode(x % c.r, c.r, c.fr_limbs)


def decode_fr(c: CurveParams, b: bytes) -> int:
    return mont_decode(b, c.r, c.fr_limbs)


def encode_fp(c: CurveParams, x: int) -> bytes:
    return mont_encode(x % c.p, c.p, c.fp_limbs)


def encode_point(c: CurveParams, P, g2: bool) -> bytes:
    """gnark G1Affine {X,Y} / G2Affine {X:{A0,A1}, Y:{A0,A1}}; infinity = zeros."""
    n = 8 * c.fp_limbs
    if P is None:
        return bytes((4 if g2 else 2) * n)
    if g2:
        (x0, x1), (y0, y1) = P
        return encode_fp(c, x0) + encode_fp(c, x1) + encode_fp(c, y0) + encode_fp(c, y1)
    return encode_fp(c, P[0]) + encode_fp(c, P[1])


def decode_point(c: CurveParams, b: bytes, g2: bool):
    n = 8 * c.fp_limbs
    if not any(b):
        return None
    vals = [mont_decode(b[i * n:(i + 1) * n], c.p, c.fp_limbs) for i in range(4 if g2 else 2)]
    if g2:
        return ((vals[0], vals[1]), (vals[2], vals[3]))
    return (vals[0], vals[1])


# ----------------------------------------------------------------------------
# NTT with gnark-crypto fft.Domain semantics
# ----------------------------------------------------------------------------


def bitrev(i: int, logn: int) -> int:
    return int(format(i, "0%db" % logn)[::-1], 2) if logn else 0


def bit_reverse(a):
    n = len(a)
    logn = n.bit_length() - 1
    return [a[bitrev(i, logn)] for i in range(n)]


def domain_generator(c: CurveParams, n: int) -> int:
    logn = n.bit_length() - 1
    assert 1 << logn == n and logn <= c.two_adicity
    return pow(c.omega_max, 1 << (c.two_adicity - logn), c.r)


def _ntt_natural(c: CurveParams, coeffs, omega):
    """evaluations[i] = sum_j coeffs[j] * omega^(i*j), natural order in/out (radix-2)."""
    r = c.r
    n = len(coeffs)
    if n == 1:
        return [coeffs[0] % r]
    even = _ntt_natural(c, coeffs[0::2], omega * omega % r)
    odd = _ntt_natural(c, coeffs[1::2], omega * omega % r)
    out = [0] * n
    w = 1
    for i in range(n // 2):
        t = w * odd[i] % r
        out[i] = (even[i] + t) % r
        out[i + n // 2] = (even[i] - t) % r
        w = w * omega % r
    return out


def fft(c: CurveParams, a, decimation: str, coset: bool = False):
    """Domain.FFT: coefficients -> evaluations at omega^i (g*omega^i on coset).
    DIF: natural in, bit-reversed out.  DIT: bit-reversed in, natural out."""
    n = len(a)
    r = c.r
    coeffs = list(a) if decimation == "DIF" else bit_reverse(a)
    if coset:
        g = c.coset_gen
        coeffs = [x * pow(g, j, r) % r for j, x in enumerate(coeffs)]
    ev = _ntt_natural(c, coeffs, domain_generator(c, n))
    return bit_reverse(ev) if decimation == "DIF" else ev


def fft_inverse(c: CurveParams, a, decimation: str, coset: bool = False):
    """Domain.FFTInverse: evaluations -> coefficients (scaled by 1/n).
    DIF: natural in, bit-reversed out.  DIT: bit-reversed in, natural out."""
    n = len(a)
    r = c.r
    ev = list(a) if decimation == "DIF" else bit_reverse(a)
    winv = pow(domain_generator(c, n), -1, r)
    coeffs = _ntt_natural(c, ev, winv)
    ninv = pow(n, -1, r)
    coeffs = [x * ninv % r for x in coeffs]
    if coset:
        ginv = pow(c.coset_gen, -1, r)
        coeffs = [x * pow(ginv, j, r) % r for j, x in enumerate(coeffs)]
    return bit_reverse(coeffs) if decimation == "DIF" else coeffs


def compute_h(c: CurveParams, a, b, cc, n: int):
    """prove.go:356-399.  Returns h in BIT-REVERSED coefficient order (len n)."""
    r = c.r
    pad = [0] * (n - len(a))
    a = list(a) + pad
    b = list(b) + pad
    cc = list(cc) + pad
    a = fft_inverse(c, a, "DIF")
    b = fft_inverse(c, b, "DIF")
    cc = fft_inverse(c, cc, "DIF")
    a = fft(c, a, "DIT", coset=True)
    b = fft(c, b, "DIT", coset=True)
    cc = fft(c, cc, "DIT", coset=True)
    den = pow((pow(c.coset_gen, n, r) - 1) % r, -1, r)
    h = [(x * y - z) * den % r for x, y, z in zip(a, b, cc)]
    return fft_inverse(c, h, "DIF", coset=True)


def filter_heap(slice_, first_index: int, to_remove):
    """prove.go:331-354 semantics: drop positions whose absolute index (i +
    first_index) appears in to_remove (duplicates allowed)."""
    rm = set(to_remove)
    if not to_remove:
        return list(slice_)
    return [v for i, v in enumerate(slice_) if i + first_index not in rm]


# ----------------------------------------------------------------------------
# deterministic synthetic inputs
# ----------------------------------------------------------------------------


def random_scalars(c: CurveParams, n: int, seed: int):
    rng = random.Random(seed)
    return [rng.randrange(c.r) for _ in range(n)]


def random_points(c: CurveParams, n: int, seed: int, g2: bool = False):
    G = Group(c, g2)
    rng = random.Random(seed)
    gen = G.generator()
    return [G.mul(gen, rng.randrange(1, c.r)) for _ in range(n)]


# ----------------------------------------------------------------------------
# Groth16 (small circuits only) -- setup.go:85-349 / prove.go:62-325 without
# BSB22 commitments.  Constraints: list of (L, R, O) sparse rows [(wire, coeff)].
# ----------------------------------------------------------------------------


def g16_setup(c: CurveParams, cons, nb_wires: int, nb_public: int, toxic):
    t, alpha, beta, gamma, delta = (x % c.r for x in toxic)
    r = c.r
    nc = len(cons)
    n = 1
    while n < nc:
        n <<= 1
    w = domain_generator(c, n)
    A, B, C = [0] * nb_wires, [0] * nb_wires, [0] * nb_wires
    tn1 = (pow(t, n, r) - 1) % r
    ninv = pow(n, -1, r)
    for j, (L, Rr, O) in enumerate(cons):
        wj = pow(w, j, r)
        lag = wj * tn1 * ninv * pow((t - wj) % r, -1, r) % r   # L_j(t)
        for wi, co in L:
            A[wi] = (A[wi] + co * lag) % r
        for wi, co in Rr:
            B[wi] = (B[wi] + co * lag) % r
        for wi, co in O:
            C[wi] = (C[wi] + co * lag) % r
    dinv = pow(delta, -1, r)
    G1, G2 = Group(c, False), Group(c, True)
    g1, g2 = c.g1, c.g2
    K = [(beta * A[i] + alpha * B[i] + C[i]) * dinv % r for i in range(nb_public, nb_wires)]
    Z = [(pow(t, i, r) * tn1 * dinv) % r for i in range(n)]
    infA = [a == 0 for a in A]
    infB = [b == 0 for b in B]
    Zp = [G1.mul(g1, z) for z in Z]
    logn = n.bit_length() - 1
    Zp = [Zp[bitrev(i, logn)] for i in range(n)][: n - 1]
    return {
        "n": n, "nb_wires": nb_wires, "nb_public": nb_public,
        "g1_alpha": G1.mul(g1, alpha), "g1_beta": G1.mul(g1, beta), "g1_delta": G1.mul(g1, delta),
        "g1_A": [G1.mul(g1, a) for a in A if a], "g1_B": [G1.mul(g1, b) for b in B if b],
        "g1_Z": Zp, "g1_K": [G1.mul(g1, k) for k in K],
        "g2_beta": G2.mul(g2, beta), "g2_delta": G2.mul(g2, delta),
        "g2_B": [G2.mul(g2, b) for b in B if b],
        "infA": infA, "infB": infB,
    }


def g16_prove(c: CurveParams, pk, wires, a, b, cc, r_: int, s_: int):
    G1, G2 = Group(c, False), Group(c, True)
    rr = c.r
    n = pk["n"]
    h = compute_h(c, a, b, cc, n)
    wA = [v for v, inf in zip(wires, pk["infA"]) if not inf]
    wB = [v for v, inf in zip(wires, pk["infB"]) if not inf]
    kr = (-r_ * s_) % rr
    delta = pk["g1_delta"]
    ar = G1.add(G1.add(G1.msm(wA, pk["g1_A"]), pk["g1_alpha"]), G1.mul(delta, r_))
    bs1 = G1.add(G1.add(G1.msm(wB, pk["g1_B"]), pk["g1_beta"]), G1.mul(delta, s_))
    krs = G1.add(G1.msm(wires[pk["nb_public"]:], pk["g1_K"]), G1.mul(delta, kr))
    krs = G1.add(krs, G1.msm(h[: n - 1], pk["g1_Z"]))
    krs = G1.add(krs, G1.mul(ar, s_) if ar else None)
    krs = G1.add(krs, G1.mul(bs1, r_) if bs1 else None)
    bs = G2.add(G2.add(G2.msm(wB, pk["g2_B"]), G2.mul(pk["g2_delta"], s_)), pk["g2_beta"])
    return ar, bs, krs


# ----------------------------------------------------------------------------
# BSB22 commitments (prove.go:82-139; verify.go:86-121; constraint/commitment.go)
#
# The arithmetic lives in gnark-crypto (not vendored): pedersen.ProvingKey
# {Basis, BasisExpSigma} with Commit = MultiExp(Basis, v) and ProveKnowledge =
# MultiExp(BasisExpSigma, v); G1Affine.Fold(points, c) = sum_i c^i points[i];
# fr.Hash(msg, dst, count) = RFC 9380 hash_to_field: expand_message_xmd with
# SHA-256, L = 16 + ceil(Bits / 8) = 48 bytes per element, big-endian mod r;
# hash_to_field.New(dst) is the hash.Hash whose Sum is fr.Hash(msg, dst, 1)[0]
# as 32 big-endian bytes; G1Affine.Marshal is the UNCOMPRESSED encoding
# (verify.go:88 sizes its buffer with SizeOfG1AffineUncompressed).  Pinned by
# RFC 9380's expand_message_xmd test vectors (tests/test_oracle.py) and by the
# exponent-form verification of whole proofs (verify.go's pairing equation +
# pedersen.BatchVerifyMultiVk, restated for a setup whose toxic waste is known).
# ----------------------------------------------------------------------------
COMMITMENT_DST = b"bsb22-commitment"  # constraint.CommitmentDst (constraint/commitment.go:7)
POK_DST = b"G16-BSB22"                # prove.go:133, verify.go:110


def expand_message_xmd(msg: bytes, dst: bytes, len_in_bytes: int) -> bytes:
    """RFC 9380 section 5.3.1 with H = SHA-256 (b_in_bytes 32, s_in_bytes 64)."""
    import hashlib
    ell = (len_in_bytes + 31) // 32
    assert ell <= 255 and len(dst) <= 255 and len_in_bytes < 65536
    dst_prime = dst + bytes([len(dst)])
    msg_prime = bytes(64) + msg + len_in_bytes.to_bytes(2, "big") + b"\x00" + dst_prime
    b0 = hashlib.sha256(msg_prime).digest()
    bi = hashlib.sha256(b0 + b"\x01" + dst_prime).digest()
    out = bi
    for i in range(2, ell + 1):
        bi = hashlib.sha256(bytes(x ^ y for x, y in zip(b0, bi)) + bytes([i]) + dst_prime).digest()
        out += bi
    return out[:len_in_bytes]


def fr_byte_len(c: CurveParams) -> int:
    """(fr.Bits - 1) / 8 + 1 (prove.go:98)."""
    return (c.r.bit_length() - 1) // 8 + 1


def hash_to_fr(c: CurveParams, msg: bytes, dst: bytes, count: int = 1):
    """gnark-crypto fr.Hash: count elements of RFC 9380 hash_to_field."""
    L = 16 + fr_byte_len(c)
    u = expand_message_xmd(msg, dst, count * L)
    return [int.from_bytes(u[i * L:(i + 1) * L], "big") % c.r for i in range(count)]


def marshal_fr(c: CurveParams, x: int) -> bytes:
    """fr.Element.Marshal: canonical value, big-endian."""
    return (x % c.r).to_bytes(fr_byte_len(c), "big")


def marshal_g1(c: CurveParams, P) -> bytes:
    """G1Affine.Marshal (RawBytes, uncompressed): X || Y big-endian; infinity is
    all zero with the uncompressed-infinity flag where the curve has one
    (BLS12-377: 0b010 << 5 in the top byte; BN254: none)."""
    n = 8 * c.fp_limbs
    if P is None:
        out = bytearray(2 * n)
        if c.name != "bn254":
            out[0] = 0b010 << 5
        return bytes(out)
    return P[0].to_bytes(n, "big") + P[1].to_bytes(n, "big")


def serialize_commitment(private_commitment: bytes, public_committed, field_byte_len: int) -> bytes:
    """constraint.SerializeCommitment (constraint/commitment.go:70-82)."""
    return private_commitment + b"".join(int(v).to_bytes(field_byte_len, "big") for v in public_committed)


def bsb22_commitment_value(c: CurveParams, D, hashed_values) -> int:
    """The commitment wire's value from the overridden BSB22 hint (prove.go:83-108):
    hash_to_field(Marshal(D) || public/commitment-committed values)."""
    msg = serialize_commitment(marshal_g1(c, D), [v % c.r for v in hashed_values], fr_byte_len(c))
    return hash_to_fr(c, msg, COMMITMENT_DST, 1)[0]


def pok_challenge(c: CurveParams, commitment_wire_values) -> int:
    """prove.go:129-136: fr.Hash(concat Marshal(w[CommitmentIndex_i]), "G16-BSB22", 1)[0]."""
    return hash_to_fr(c, b"".join(marshal_fr(c, v) for v in commitment_wire_values), POK_DST, 1)[0]


def fold_points(c: CurveParams, points, coeff: int):
    """G1Affine.Fold (prove.go:137): sum_i coeff^i points[i]."""
    G = Group(c, False)
    acc, e = None, 1
    for P in points:
        acc = G.add(acc, G.mul(P, e) if P else None)
        e = e * coeff % c.r
    return acc
