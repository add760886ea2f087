"""Element-wise parity of the device field / curve primitives (gm_test_field_op,
gm_test_point_op) vs the big-integer oracle (oracle/pyref.py)."""
import random

import pytest

import pyref

pytestmark = pytest.mark.gpu

N = 64


def _fp_vals(c, n, seed, edge=True):
    rng = random.Random(seed)
    v = [rng.randrange(c.p) for _ in range(n)]
    if edge:
        v[:6] = [0, 1, 2, c.p - 1, c.p - 2, (c.p - 1) // 2]
    return v


def _enc(c, vals, modulus, limbs):
    return b"".join(pyref.mont_encode(x, modulus, limbs) for x in vals)


def _dec(c, b, modulus, limbs):
    w = 8 * limbs
    return [pyref.mont_decode(b[i:i + w], modulus, limbs) for i in range(0, len(b), w)]


@pytest.mark.parametrize("cname", ["bn254", "bls12377"])
@pytest.mark.parametrize("kind", [0, 1])
def test_field_ops(gm_ctx, cname, kind):
    c = pyref.CURVES[cname]
    mod, limbs = (c.r, c.fr_limbs) if kind == 0 else (c.p, c.fp_limbs)
    a = [x % mod for x in _fp_vals(c, N, 1)]
    b = [x % mod for x in _fp_vals(c, N, 2)][::-1]
    A, B = _enc(c, a, mod, limbs), _enc(c, b, mod, limbs)
    ref = {
        0: [x * y % mod for x, y in zip(a, b)],
        1: [(x + y) % mod for x, y in zip(a, b)],
        2: [(x - y) % mod for x, y in zip(a, b)],
        3: [(-x) % mod for x in a],
        4: [pow(x, mod - 2, mod) for x in a],
        5: [x * x % mod for x in a],
    }
    for op, exp in ref.items():
        got = _dec(c, gm_ctx.test_field_op(cname, kind, op, A, B), mod, limbs)
        assert got == exp, (cname, kind, op)
        # outputs must be fully reduced (canonical Montgomery words)
        assert gm_ctx.test_field_op(cname, kind, op, A, B) == _enc(c, exp, mod, limbs)


@pytest.mark.parametrize("cname", ["bn254", "bls12377"])
def test_fp2_ops(gm_ctx, cname):
    c = pyref.CURVES[cname]
    F = pyref.F2(c)
    a = list(zip(_fp_vals(c, N, 3), _fp_vals(c, N, 4)))
    b = list(zip(_fp_vals(c, N, 5), _fp_vals(c, N, 6)))[::-1]
    enc = lambda v: b"".join(pyref.encode_fp(c, x0) + pyref.encode_fp(c, x1) for x0, x1 in v)
    A, B = enc(a), enc(b)
    ref = {0: [F.mul(x, y) for x, y in zip(a, b)], 1: [F.add(x, y) for x, y in zip(a, b)],
           2: [F.sub(x, y) for x, y in zip(a, b)], 3: [F.neg(x) for x in a],
           4: [F.inv(x) if not F.is_zero(x) else (0, 0) for x in a], 5: [F.mul(x, x) for x in a]}
    for op, exp in ref.items():
        assert gm_ctx.test_field_op(cname, 2, op, A, B) == enc(exp), (cname, op)


@pytest.mark.parametrize("cname", ["bn254", "bls12377"])
@pytest.mark.parametrize("g2", [False, True])
def test_point_ops(gm_ctx, cname, g2):
    c = pyref.CURVES[cname]
    G = pyref.Group(c, g2)
    n = 16
    P = pyref.random_points(c, n, 11, g2)
    Q = pyref.random_points(c, n, 12, g2)
    P[0] = None
    Q[1] = None
    Q[2] = P[2]
    Q[3] = G.neg(P[3])
    enc = lambda v: b"".join(pyref.encode_point(c, x, g2) for x in v)
    A, B = enc(P), enc(Q)
    exp = {0: [G.add(p, q) for p, q in zip(P, Q)], 1: [G.add(p, p) for p in P],
           2: [G.add(p, q) for p, q in zip(P, Q)], 3: [G.mul(p, 1000003) if p else None for p in P]}
    for op, e in exp.items():
        assert gm_ctx.test_point_op(cname, g2, op, A, B) == enc(e), (cname, g2, op)
