"""NTT parity: HIP multi-pass radix-2 NTT (gm_ntt; replaces iciclegnark
NttOnDevice / INttOnDevice, icicle.go:489-502) vs the oracle's restatement of
gnark-crypto fft.Domain.FFT / FFTInverse (prove.go:372-378,396), all four
orderings x coset.  Bit-exact."""
import itertools

import numpy as np
import pytest

import pyref

pytestmark = pytest.mark.gpu

MODES = list(itertools.product([0, 1], [0, 1], [0, 1]))  # inverse, dit, coset


@pytest.mark.parametrize("cname", ["bn254", "bls12377"])
@pytest.mark.parametrize("logn", [0, 1, 2, 3, 4, 5, 8, 9, 10, 11, 12, 16, 17])
def test_ntt_modes_vs_oracle(gm_ctx, oracle, cname, logn):
    n = 1 << logn
    X = gm_ctx.random_scalars(cname, n, seed=0x5EED0003 + logn)
    xb = X.to_host()
    for inverse, dit, coset in MODES:
        X.write(xb)
        gm_ctx.ntt(cname, X, n, inverse, dit, coset)
        got = X.to_host()
        exp = oracle.fft(cname, xb, inverse, dit, coset)
        assert got == exp, (cname, logn, inverse, dit, coset)
    X.free()


@pytest.mark.parametrize("cname", ["bn254", "bls12377"])
def test_ntt_small_vs_pyref(gm_ctx, cname):
    c = pyref.CURVES[cname]
    n = 16
    vals = pyref.random_scalars(c, n, 4)
    xb = b"".join(pyref.encode_fr(c, v) for v in vals)
    X = gm_ctx.copy_to_device(xb)
    for inverse, dit, coset in MODES:
        X.write(xb)
        gm_ctx.ntt(cname, X, n, inverse, dit, coset)
        got = X.to_host()
        fn = pyref.fft_inverse if inverse else pyref.fft
        exp = fn(c, vals, "DIT" if dit else "DIF", bool(coset))
        assert [pyref.decode_fr(c, got[32 * i:32 * i + 32]) for i in range(n)] == exp
    X.free()


@pytest.mark.parametrize("logn", [20, 22])
def test_ntt_roundtrip_large(gm_ctx, logn):
    """Size-independent property at large n: INTT(DIT) o NTT(DIF) = id, also on coset."""
    n = 1 << logn
    X = gm_ctx.random_scalars("bn254", n, seed=logn)
    xb = X.to_host()
    for coset in (0, 1):
        gm_ctx.ntt("bn254", X, n, 0, 0, coset)
        assert X.to_host() != xb
        gm_ctx.ntt("bn254", X, n, 1, 1, coset)
        assert X.to_host() == xb
    X.free()


@pytest.mark.parametrize("cname", ["bn254", "bls12377"])
@pytest.mark.parametrize("length,n", [(3, 4), (13, 16), (1000, 1024), ((1 << 15) - 5, 1 << 15)])
def test_compute_h_vs_oracle(gm_ctx, oracle, cname, length, n):
    A = gm_ctx.random_scalars(cname, n, seed=1 + length)
    B = gm_ctx.random_scalars(cname, n, seed=2 + length)
    C = gm_ctx.random_scalars(cname, n, seed=3 + length)
    ab, bb, cb = (x.to_host(32 * length) for x in (A, B, C))
    exp = oracle.compute_h(cname, ab, bb, cb, n)
    gm_ctx.compute_h(cname, A, B, C, length, n)
    assert A.to_host() == exp
    for x in (A, B, C):
        x.free()


def test_reverse_and_poly_ops(gm_ctx):
    c = pyref.BN254
    n = 64
    vals = pyref.random_scalars(c, 3 * n, 9)
    enc = lambda v: b"".join(pyref.encode_fr(c, x) for x in v)
    A, B, C = (gm_ctx.copy_to_device(enc(vals[i * n:(i + 1) * n])) for i in range(3))
    den = 0x1234567
    gm_ctx.poly_ops("bn254", A, B, C, n, pyref.encode_fr(c, den))
    got = A.to_host()
    exp = [(vals[i] * vals[n + i] - vals[2 * n + i]) * den % c.r for i in range(n)]
    assert [pyref.decode_fr(c, got[32 * i:32 * i + 32]) for i in range(n)] == exp
    gm_ctx.reverse_scalars("bn254", A, n)
    got2 = A.to_host()
    assert [pyref.decode_fr(c, got2[32 * i:32 * i + 32]) for i in range(n)] == pyref.bit_reverse(exp)
    for x in (A, B, C):
        x.free()
