"""Derives the BN254 G1 GLV constants of csrc/msm_impl.hpp (GlvBn254) and checks
them against the oracle's group law (test infrastructure, not product code).

phi(x, y) = (beta x, y) = [lambda] P; short basis of the lattice
{(a, b): a + b lambda = 0 mod r} from the extended Euclid on (r, lambda);
c1 = floor(k g1 / 2^384), c2 = floor(k g2 / 2^384) with g1 = floor(2^384 b2 / r),
g2 = floor(2^384 |b1| / r); k1 = k - c1 a1 - c2 a2 in [0, 2^127),
k2 = c1 |b1| - c2 b2 in (-2^127, 2^127).  Run: python tools/glv_constants.py
"""
import os
import random
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "oracle"))
import pyref  # noqa: E402

SH = 384


def cube_roots(m):
    for g in range(2, 100):
        w = pow(g, (m - 1) // 3, m)
        if w != 1:
            return [w, w * w % m]


def short_basis(r, lam):
    """Two short vectors (a, b) with a + b lam = 0 mod r (GLV, sec. 4)."""
    r0, r1, t0, t1 = r, lam, 0, 1
    hist = [(r0, t0), (r1, t1)]
    while r1 * r1 >= r:
        q = r0 // r1
        r0, r1 = r1, r0 - q * r1
        t0, t1 = t1, t0 - q * t1
        hist.append((r1, t1))
    rm, tm = hist[-2]
    rm1, tm1 = hist[-1]
    q = r0 // r1
    rn, tn = r0 - q * r1, t0 - q * t1
    v1 = (rm1, -tm1)
    v2 = (rm, -tm) if rm * rm + tm * tm <= rn * rn + tn * tn else (rn, -tn)
    return v1, v2


def derive():
    c = pyref.BN254
    p, r = c.p, c.r
    G = pyref.Group(c, False)
    P0 = G.generator()
    lam = beta = None
    for l_ in cube_roots(r):
        for b_ in cube_roots(p):
            if G.mul(P0, l_) == (b_ * P0[0] % p, P0[1]):
                lam, beta = l_, b_
    (a1, b1), (a2, b2) = short_basis(r, lam)
    assert a1 * b2 - a2 * b1 == r and a1 > 0 and a2 > 0 and b1 < 0 and b2 > 0
    assert a2 == -b1
    g1 = (b2 << SH) // r
    g2 = ((-b1) << SH) // r
    return dict(p=p, r=r, lam=lam, beta=beta, a1=a1, b1=b1, a2=a2, b2=b2, g1=g1, g2=g2)


def split(k, d):
    M = (1 << 128) - 1
    c1 = (k * d["g1"]) >> SH
    c2 = (k * d["g2"]) >> SH
    k1 = (k - c1 * d["a1"] - c2 * d["a2"]) & M
    k2 = (c1 * (-d["b1"]) - c2 * d["b2"]) & M
    k2 = k2 - (1 << 128) if k2 >> 127 else k2
    return k1, k2


def derive_bls12377():
    """BLS12-377: lambda = x^2 - 1 (x = 0x8508c00000000001 the curve seed) is a
    cube root of unity of r with lambda^2 < r < (lambda + 1)^2, so the split is a
    plain division: k2 = floor(k / lambda) < 2^127, k1 = k - k2 lambda < lambda
    (both unsigned).  Device: q = floor(k g / 2^384), g = floor(2^384 / lambda),
    undershoots k / lambda by < 1, then one conditional correction."""
    c = pyref.BLS12_377 if hasattr(pyref, "BLS12_377") else pyref.CURVES["bls12377"]
    p, r = c.p, c.r
    x = 0x8508c00000000001
    lam = x * x - 1
    assert (lam * lam + lam + 1) % r == 0 and lam < (1 << 127) and lam * lam < r < (lam + 1) ** 2
    G1, G2 = pyref.Group(c, False), pyref.Group(c, True)
    P, Q = G1.generator(), G2.generator()
    b1 = [b for b in cube_roots(p) if G1.mul(P, lam) == (b * P[0] % p, P[1])]
    LQ = G2.mul(Q, lam)
    b2 = [b for b in cube_roots(p) if LQ == ((Q[0][0] * b % p, Q[0][1] * b % p), Q[1])]
    assert len(b1) == 1 and len(b2) == 1 and b2[0] == b1[0] * b1[0] % p
    return dict(p=p, r=r, lam=lam, beta=b1[0], beta_g2=b2[0], g=(1 << SH) // lam)


def split_bls12377(k, d):
    M = (1 << 128) - 1
    q = (k * d["g"]) >> SH
    k1 = (k - q * d["lam"]) & M
    if k1 >= d["lam"]:
        k1 -= d["lam"]
        q += 1
    return k1, q


def main_bls12377():
    d = derive_bls12377()
    r, lam = d["r"], d["lam"]
    rng = random.Random(8)
    specials = [0, 1, 2, r - 1, r - 2, lam, lam - 1, lam + 1, lam * lam, lam * lam - 1, lam * lam + lam,
                r - lam, (r - 1) // 2, 1 << 252]
    for t in range(200000):
        k = specials[t] if t < len(specials) else rng.randrange(r)
        k1, k2 = split_bls12377(k, d)
        assert 0 <= k1 < lam and 0 <= k2 < (1 << 127) and k1 + k2 * lam == k
    c = pyref.CURVES["bls12377"]
    G1 = pyref.Group(c, False)
    for P in pyref.random_points(c, 3, 12):
        assert G1.mul(P, lam) == (d["beta"] * P[0] % d["p"], P[1])

    def l64(x, n):
        return ", ".join("0x%016xull" % ((x >> (64 * i)) & (2 ** 64 - 1)) for i in range(n))

    def r29(v):
        vi = v * (1 << (29 * 14)) % d["p"]
        return ", ".join("0x%08xu" % ((vi >> (29 * i)) & (2 ** 29 - 1)) for i in range(14))
    print("BLS12-377 g", l64(d["g"], 5))
    print("BLS12-377 lambda", l64(lam, 2))
    print("BLS12-377 beta29 (G1)", r29(d["beta"]))
    print("BLS12-377 beta29 (G2 twist, beta^2)", r29(d["beta_g2"]))
    print("BLS12-377 split checked on 200000 scalars; phi checked on G1 and G2 generators")


def main():
    d = derive()
    r, lam = d["r"], d["lam"]
    specials = [0, 1, 2, r - 1, r - 2, lam, r - lam, lam + 1, lam - 1, d["a1"], d["b2"], r - d["b2"],
                (r - 1) // 2, (r + 1) // 2, 1 << 253]
    rng = random.Random(7)
    for t in range(200000):
        k = specials[t] if t < len(specials) else rng.randrange(r)
        k1, k2 = split(k, d)
        assert 0 <= k1 < (1 << 127) and abs(k2) < (1 << 127)
        assert (k1 + k2 * lam - k) % r == 0
    # group-law check of phi on random points
    G = pyref.Group(pyref.BN254, False)
    for P in pyref.random_points(pyref.BN254, 4, 11):
        assert G.mul(P, lam) == (d["beta"] * P[0] % d["p"], P[1])

    def l64(x, n):
        return ", ".join("0x%016xull" % ((x >> (64 * i)) & (2 ** 64 - 1)) for i in range(n))
    bi = d["beta"] * (1 << 261) % d["p"]
    print("g1", l64(d["g1"], 5))
    print("g2", l64(d["g2"], 4))
    print("a1", l64(d["a1"], 2), " a2=|b1|", l64(d["a2"], 1), " b2", l64(d["b2"], 2))
    print("beta29", ", ".join("0x%08xu" % ((bi >> (29 * i)) & (2 ** 29 - 1)) for i in range(9)))
    print("split checked on 200000 scalars; phi checked on 4 points")


if __name__ == "__main__":
    main()
    main_bls12377()
