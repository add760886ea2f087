"""Replays backend/groth16/bn254/icicle/icicle.go call for call through the
iciclegnark-semantics C-ABI (gm_icicle_*, gm_msm, gm_reverse_scalars, gm_free)
-- the binding INTEGRATION.md §2 gives the Go shim -- and checks that the
reference's own call sequence, ownership included, yields the oracle's h and
proof:

  setupDevicePointers  icicle.go:31-130   (den vector, twiddle handles, coset tables, points)
  computeH             icicle.go:453-513  (INtt -> Ntt(coset) -> free, PolyOps, coset INtt,
                                           free a/b/c, ReverseScalars)
  Prove device block   icicle.go:231-412  (compaction + H2D, 4 G1 MSMs, 1 G2 MSM, frees)

The host finishing adds (AddMixed, ScalarMultiplication, FromJacobian) stay in
Go / gnark-crypto in the reference; here pyref's group arithmetic plays them.
"""
import numpy as np
import pytest

import pyref
import r1cs as R

pytestmark = pytest.mark.gpu

TOXIC = [0x11D5A2B3C4D5E6F708192A3B4C5D6E7F8091A2B3C4D5E6F708192A3B4C5D6,
         0x22E6B3C4D5E6F708192A3B4C5D6E7F8091A2B3C4D5E6F708192A3B4C5D6E7,
         0x33F7C4D5E6F708192A3B4C5D6E7F8091A2B3C4D5E6F708192A3B4C5D6E7F8,
         0x40A8D5E6F708192A3B4C5D6E7F8091A2B3C4D5E6F708192A3B4C5D6E7F809,
         0x51B9E6F708192A3B4C5D6E7F8091A2B3C4D5E6F708192A3B4C5D6E7F8091A]


class DevicePk:
    """pk.deviceInfo as setupDevicePointers (icicle.go:31-130) fills it."""

    def __init__(self, ctx, cname, pk, n, g1b):
        c = pyref.CURVES[cname]
        enc = lambda v: R.encode_vec(cname, v)
        self.bufs = []
        keep = lambda b: (self.bufs.append(b), b)[1]
        g = c.coset_gen
        # CosetTableInv / CosetTable (icicle.go:44,47): g^-i, g^i
        gi = pow(g, -1, c.r)
        self.coset_inv = keep(ctx.copy_to_device(enc([pow(gi, i, c.r) for i in range(n)])))
        self.coset = keep(ctx.copy_to_device(enc([pow(g, i, c.r) for i in range(n)])))
        # Den (icicle.go:50-65): n copies of 1 / (g^n - 1)
        den = pow((pow(g, n, c.r) - 1) % c.r, -1, c.r)
        self.den = keep(ctx.copy_to_device(enc([den]) * n))
        # Twiddles (icicle.go:68-80)
        self.tw_inv = keep(ctx.icicle_generate_twiddle_factors(cname, n, True))
        self.tw = keep(ctx.icicle_generate_twiddle_factors(cname, n, False))
        # G1 A, B; K minus its infinity points (InfinityPointIndicesK); Z; G2 B (icicle.go:84-127)
        self.A = keep(ctx.copy_points_to_device(cname, pk["g1_A"]))
        self.B = keep(ctx.copy_points_to_device(cname, pk["g1_B"]))
        K = np.frombuffer(bytes(pk["g1_K"]), np.uint8).reshape(-1, g1b)
        inf = np.all(K == 0, axis=1)
        self.inf_k = [int(i) for i in np.nonzero(inf)[0]]
        self.K = keep(ctx.copy_points_to_device(cname, K[~inf].tobytes()))
        self.nbK = int((~inf).sum())
        self.Z = keep(ctx.copy_points_to_device(cname, pk["g1_Z"]))
        self.B2 = keep(ctx.copy_points_to_device(cname, pk["g2_B"], g2=True))

    def free(self):
        for b in self.bufs:
            b.free()


def compute_h_replay(ctx, cname, dpk, a, b, cc, n):
    """icicle.go:453-513, call for call; returns the device pointer h."""
    pad = lambda v: v + bytes(32 * n - len(v))
    a_d, b_d, c_d = (ctx.copy_to_device(pad(v)) for v in (a, b, cc))   # :466-480
    for d in (a_d, b_d, c_d):                                          # :482-495
        a_intt_d = ctx.icicle_intt_on_device(cname, d, n, False)
        ctx.icicle_ntt_on_device(cname, d, a_intt_d, n, True)
        a_intt_d.free()                                                # FreeDevicePointer(a_intt_d)
    ctx.icicle_poly_ops(cname, a_d, b_d, c_d, dpk.den, n)              # :500
    h = ctx.icicle_intt_on_device(cname, a_d, n, True)                 # :502
    for d in (a_d, b_d, c_d):                                          # :504-508
        d.free()
    ctx.reverse_scalars(cname, h, n)                                   # :510
    return h


@pytest.mark.parametrize("k", [15, 1023])
def test_icicle_call_sequence_replay(gm_ctx, oracle, k):
    import gnark_mi355x as gm
    cname = "bn254"
    c = pyref.CURVES[cname]
    G1, G2 = pyref.Group(c, False), pyref.Group(c, True)
    g1b = gm.point_bytes(cname, False)
    r1, W = R.squaring_chain(k, cname, x=7)
    n = r1.domain_size
    enc = lambda v: R.encode_vec(cname, v)
    tox = enc([t % c.r for t in TOXIC])
    pk = oracle.g16_setup(cname, r1, tox)
    a, b, cc = (enc(v) for v in r1.solve_abc(W))
    rr, ss = 0x1F2E3D4C5B6A, 0x0A1B2C3D4E5F
    exp = oracle.g16_prove(cname, pk, r1.nb_public, enc(W), a, b, cc, enc([rr]), enc([ss]))

    dpk = DevicePk(gm_ctx, cname, pk, n, g1b)
    try:
        h = compute_h_replay(gm_ctx, cname, dpk, a, b, cc, n)
        assert h.to_host() == oracle.compute_h(cname, a, b, cc, n)       # bit-reversed h

        # compaction + H2D (icicle.go:231-278)
        infA, infB = np.asarray(pk["infA"]), np.asarray(pk["infB"])
        wA = enc([w for i, w in enumerate(W) if not infA[i]])
        wB = enc([w for i, w in enumerate(W) if not infB[i]])
        wA_d, wB_d = gm_ctx.copy_to_device(wA), gm_ctx.copy_to_device(wB)
        nA, nB = len(wA) // 32, len(wB) // 32
        dec1 = lambda jac: pyref.decode_point(c, gm.jac_to_affine(cname, False, jac), False)
        dec2 = lambda jac: pyref.decode_point(c, gm.jac_to_affine(cname, True, jac), True)
        pt = lambda key, g2=False: pyref.decode_point(c, bytes(pk[key]), g2)
        # r, s, kr and the deltas (icicle.go:280-295)
        kr = -rr * ss % c.r
        delta = pt("g1_delta")
        deltas = [G1.mul(delta, x) for x in (rr, ss, kr)]
        # computeBS1 / computeAR1 (icicle.go:299-324)
        bs1 = G1.add(G1.add(dec1(gm_ctx.msm_on_device(wB_d, dpk.B, nB)), pt("g1_beta")), deltas[1])
        ar = G1.add(G1.add(dec1(gm_ctx.msm_on_device(wA_d, dpk.A, nA)), pt("g1_alpha")), deltas[0])
        # computeKRS (icicle.go:326-375): Z MSM over h[:n-1], K over the filtered wires
        krs2 = dec1(gm_ctx.msm_on_device(h, dpk.Z, n - 1))
        scalars = list(W[r1.nb_public:])
        for idx in dpk.inf_k:                      # icicle.go:343-347 (single removal per index)
            del scalars[idx]
        scalars_d = gm_ctx.copy_to_device(enc(scalars))
        krs = dec1(gm_ctx.msm_on_device(scalars_d, dpk.K, len(scalars)))
        scalars_d.free()                                                   # :356
        krs = G1.add(krs, deltas[2])
        krs = G1.add(krs, krs2)
        krs = G1.add(krs, G1.mul(ar, ss))
        krs = G1.add(krs, G1.mul(bs1, rr))
        # computeBS2 (icicle.go:377-393)
        bs = dec2(gm_ctx.msm_g2_on_device(wB_d, dpk.B2, nB))
        bs = G2.add(G2.add(bs, G2.mul(pt("g2_delta", True), ss)), pt("g2_beta", True))
        # frees (icicle.go:414-419)
        for d in (wA_d, wB_d, h):
            d.free()
    finally:
        dpk.free()
    got = (pyref.encode_point(c, ar, False), pyref.encode_point(c, bs, True), pyref.encode_point(c, krs, False))
    assert got == exp


@pytest.mark.parametrize("cname", ["bn254", "bls12377"])
@pytest.mark.parametrize("logn", [1, 4, 10, 13])
def test_icicle_ntt_semantics(gm_ctx, oracle, cname, logn):
    """INttOnDevice: natural evaluations -> fresh buffer of natural coefficients
    (input left bit-reversed); NttOnDevice: natural coefficients -> natural
    evaluations, in place or out of place; coset variants."""
    import gnark_mi355x as gm
    n = 1 << logn
    X = gm_ctx.random_scalars(cname, n, seed=logn + 99)
    xb = X.to_host()
    brev = lambda data: b"".join(data[32 * pyref.bitrev(i, logn):32 * pyref.bitrev(i, logn) + 32] for i in range(n))
    for coset in (False, True):
        X.write(xb)
        Y = gm_ctx.icicle_intt_on_device(cname, X, n, coset)
        # natural-order coefficients = bit-reverse of the DIF inverse output
        assert Y.to_host() == brev(oracle.fft(cname, xb, 1, 0, int(coset)))
        assert X.to_host() == brev(xb)
        Z = gm_ctx.malloc(32 * n)
        gm_ctx.icicle_ntt_on_device(cname, Z, Y, n, coset)
        assert Z.to_host() == brev(oracle.fft(cname, Y.to_host(), 0, 0, int(coset)))
        assert Z.to_host() == xb  # round trip
        gm_ctx.icicle_ntt_on_device(cname, Y, Y, n, coset)  # in place
        assert Y.to_host() == xb
        Y.free()
        Z.free()
    X.free()
