"""Host-only C-ABI helpers (no GPU): gm_jac_add / gm_jac_to_affine, the
finishing adds of sharded proofs (prove.go:195-305's AddMixed / ScalarMul
tail; gnark_mi355x.reduce_partials), on every edge the finishing code meets --
P + Q, P + P (the doubling branch), P + (-P), the identity on either side,
several Z representations of one point -- against the pyref group law.  Also
run under AddressSanitizer / UndefinedBehaviorSanitizer by
tools/sanitize/run.sh (host code of the library instrumented)."""
import random

import pytest

import gnark_mi355x as gm
import pyref


def _enc_f(c, g2, v):
    if g2:
        return pyref.encode_fp(c, v[0]) + pyref.encode_fp(c, v[1])
    return pyref.encode_fp(c, v)


def _jac(G, P, z):
    """gnark Jacobian bytes of affine P with Z = z (X = x z^2, Y = y z^3)."""
    c, F = G.c, G.F
    if P is None:
        return gm.jac_infinity(c.name, G.g2)
    z2 = F.mul(z, z)
    return _enc_f(c, G.g2, F.mul(P[0], z2)) + _enc_f(c, G.g2, F.mul(P[1], F.mul(z2, z))) + _enc_f(c, G.g2, z)


def _rand_z(G, rng):
    if G.g2:
        return (rng.randrange(1, G.c.p), rng.randrange(0, G.c.p))
    return rng.randrange(1, G.c.p)


@pytest.mark.parametrize("cname", ["bn254", "bls12377"])
@pytest.mark.parametrize("g2", [False, True])
def test_jac_add_and_affine_edges(cname, g2):
    c = pyref.CURVES[cname]
    G = pyref.Group(c, g2)
    rng = random.Random(7 + g2)
    gen = G.generator()
    pts = [G.mul(gen, rng.randrange(1, c.r)) for _ in range(3)]
    P, Q, R = pts
    cases = [(P, Q), (P, P), (P, G.neg(P)), (None, Q), (P, None), (None, None), (Q, R)]
    for a, b in cases:
        for _ in range(2):  # two Z representations of each operand
            ja, jb = _jac(G, a, _rand_z(G, rng)), _jac(G, b, _rand_z(G, rng))
            s = gm.jac_add(cname, g2, ja, jb)
            assert pyref.decode_point(c, gm.jac_to_affine(cname, g2, s), g2) == G.add(a, b)
    # a partial sum of many terms (the host reduction of rank partials)
    parts = [_jac(G, X, _rand_z(G, rng)) for X in pts + [G.neg(P), None]]
    got = pyref.decode_point(c, gm.jac_to_affine(cname, g2, gm.reduce_partials(cname, g2, parts)), g2)
    assert got == G.add(Q, R)
    assert gm.jac_to_affine(cname, g2, gm.jac_infinity(cname, g2)) == bytes(gm.point_bytes(cname, g2))
