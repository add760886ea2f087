"""BASELINE configs[4] PLONK/KZG path: replays, call for call, the device work
the patched BLS12-377 PLONK prover issues (integration/go/plonk_bls12377/
prove.go.diff + kzg_mi355x.go) on an SCS-sized domain, through the same C-ABI
entries the Go hook binds (gm_points_upload, gm_kzg_commit, gm_copy_to_device +
gm_ntt + gm_memcpy_d2h), against the oracle's MSM and FFT:

  deviceFor(pk)             upload pk.Kzg.G1 (canonical SRS, n + 3 points) and
                            pk.KzgLagrange.G1 (n points)
  bsb22Hint  prove.go:312   commit(Lagrange poly, KzgLagrange)
  commitToLRO :391-417 /
  commitToPolyAndBlinding :460   commit(L, R, O, Z in Lagrange form, KzgLagrange)
  divideByZH :1178-1205     FFTInverse(DIT, OnCoset) on domain1 (4n), bit-reversed in
  commitToQuotient :1154-1170    commit(h1, h2, h3 canonical, n + 2 each, Kzg)
  computeLinearizedPolynomial :718  commit(canonical, Kzg)

Beyond element-wise parity, the KZG identity ties the two SRS and the NTT
together: commit_Lagrange(p) == commit_canonical(FFTInverse(p)).
"""
import pytest

import pyref

pytestmark = pytest.mark.gpu

CNAME = "bls12377"


def _srs(oracle, gm, n, tau):
    """pk.Kzg.G1 = [tau^i] G1 (i < n + 3) and pk.KzgLagrange.G1 = [L_i(tau)] G1
    over the size-n domain (gnark's PLONK setup sizes, backend/plonk/bls12-377/
    setup.go:81-82, 119)."""
    c = pyref.CURVES[CNAME]
    r = c.r
    w = pyref.domain_generator(c, n)
    tn1 = (pow(tau, n, r) - 1) % r
    ninv = pow(n, -1, r)
    powers = [pow(tau, i, r) for i in range(n + 3)]
    lag = []
    for i in range(n):
        wi = pow(w, i, r)
        lag.append(wi * tn1 * ninv * pow((tau - wi) % r, -1, r) % r)
    enc = lambda vals: b"".join(pyref.encode_fr(c, v) for v in vals)
    gen = gm.generator(CNAME)
    canon = oracle.batch_mul_base(CNAME, False, gen, enc(powers))
    lagr = oracle.batch_mul_base(CNAME, False, gen, enc(lag))
    return canon, lagr


@pytest.mark.parametrize("logn", [6, 10])
def test_plonk_bls12377_commit_fft_replay(gm_ctx, oracle, logn):
    import gnark_mi355x as gm
    c = pyref.CURVES[CNAME]
    n = 1 << logn
    enc = lambda vals: b"".join(pyref.encode_fr(c, v) for v in vals)
    pb = gm.point_bytes(CNAME, False)
    canon, lagr = _srs(oracle, gm, n, tau=pyref.random_scalars(c, 1, 0x77)[0])
    # deviceFor(pk): both SRS resident on the device
    d_canon = gm_ctx.points_upload(CNAME, canon)
    d_lagr = gm_ctx.points_upload(CNAME, lagr)
    try:
        # bsb22Hint (:312) and commitToLRO / Z (:460): Lagrange-form commits
        for k, seed in enumerate((0x10, 0x11, 0x12, 0x13, 0x14)):
            p = pyref.random_scalars(c, n, seed)
            if k == 0:
                p[3] = 0  # committed values are sparse in the BSB22 polynomial
            pbytes = enc(p)
            got = gm_ctx.kzg_commit(CNAME, d_lagr, pbytes)
            assert got == oracle.msm(CNAME, False, pbytes, lagr), k
            # KZG identity: the same polynomial in canonical form against pk.Kzg
            # (iop ToCanonical: FFTInverse(DIF) -> bit-reversed, then ToRegular)
            X = gm_ctx.copy_to_device(pbytes)
            gm_ctx.ntt(CNAME, X, n, True, False, False)
            gm_ctx.reverse_scalars(CNAME, X, n)
            coeffs = X.to_host()
            X.free()
            brev = oracle.fft(CNAME, pbytes, True, False, False)  # FFTInverse(DIF): bit-reversed
            chunks = [brev[32 * i:32 * i + 32] for i in range(n)]
            assert coeffs == b"".join(chunks[pyref.bitrev(i, logn)] for i in range(n))
            assert gm_ctx.kzg_commit(CNAME, d_canon, coeffs) == got, k
        # divideByZH (:1178-1205): numerator on domain1's coset, bit-reversed
        # (LagrangeCoset / BitReverse) -> FFTInverse(DIT, OnCoset) -> canonical
        m = 4 * n
        num = enc(pyref.random_scalars(c, m, 0x20))
        X = gm_ctx.copy_to_device(num)  # gm.NTT: copy in, transform, copy out
        gm_ctx.ntt(CNAME, X, m, True, True, True)
        h = X.to_host()
        X.free()
        assert h == oracle.fft(CNAME, num, True, True, True)
        # commitToQuotient (:1154-1170): h1, h2, h3 of n + 2 coefficients each
        for i in range(3):
            part = h[32 * i * (n + 2):32 * (i + 1) * (n + 2)]
            got = gm_ctx.kzg_commit(CNAME, d_canon, part)
            assert got == oracle.msm(CNAME, False, part, canon[:pb * (len(part) // 32)]), i
        # computeLinearizedPolynomial (:718): a canonical polynomial of n + 2 coefficients
        lin = enc(pyref.random_scalars(c, n + 2, 0x30))
        assert gm_ctx.kzg_commit(CNAME, d_canon, lin) == oracle.msm(CNAME, False, lin, canon[:pb * (n + 2)])
        # kzg.ErrInvalidPolynomialSize: a polynomial longer than the SRS is refused
        with pytest.raises(gm.GmError):
            gm_ctx.kzg_commit(CNAME, d_lagr, enc([1] * (n + 1)))
    finally:
        d_canon.free()
        d_lagr.free()


def _quotient(r, f, fz, z):
    """(f(X) - fz) / (X - z) by synthetic division, as kzg_mi355x.go's
    quotientByXminusZ (gnark-crypto kzg's dividePolyByXminusA)."""
    f = list(f)
    f[0] = (f[0] - fz) % r
    for i in range(len(f) - 2, -1, -1):
        f[i] = (f[i] + f[i + 1] * z) % r
    return f[1:]


def _eval(r, f, z):
    acc = 0
    for a in reversed(f):
        acc = (acc * z + a) % r
    return acc


@pytest.mark.parametrize("logn", [6, 10])
def test_plonk_bls12377_openings_and_domain0_replay(gm_ctx, oracle, logn):
    """The remaining n-size MSMs and FFTs of the patched prover (prove.go.diff):
      openZ :611             kzg.Open(blindedZ, zeta*w) -> s.open: claimed value
                             (Horner), quotient (synthetic division) on the host,
                             commit(quotient, pk.Kzg) on the GPU
      batchOpening :757      kzg.BatchOpenSinglePoint -> s.batchOpen: the folded
                             polynomial sum gamma^i f_i, its quotient, GPU commit
      computeNumerator :949, :967, :1016 and :1301
                             domain0 ToCanonical (Lagrange Regular -> FFTInverse
                             DIF -> Canonical BitReverse), scaling, ToLagrange
                             (Canonical BitReverse -> FFT DIT -> Lagrange Regular)
    Each commit is checked against the oracle MSM AND against the KZG identity
    commit(q) = [(f(tau) - f(z)) / (tau - z)] G1, which pins the quotient itself
    (tau is known to the test)."""
    import gnark_mi355x as gm
    c = pyref.CURVES[CNAME]
    r = c.r
    n = 1 << logn
    enc = lambda vals: b"".join(pyref.encode_fr(c, v) for v in vals)
    dec = lambda b: [pyref.decode_fr(c, b[32 * i:32 * i + 32]) for i in range(len(b) // 32)]
    tau = pyref.random_scalars(c, 1, 0x79)[0]
    canon, _ = _srs(oracle, gm, n, tau)
    d_canon = gm_ctx.points_upload(CNAME, canon)
    gen = gm.generator(CNAME)
    G = pyref.Group(c, False)

    def commit_checked(q, what):
        got = gm_ctx.kzg_commit(CNAME, d_canon, enc(q))
        assert got == oracle.msm(CNAME, False, enc(q), canon[:gm.point_bytes(CNAME, False) * len(q)]), what
        return got

    try:
        # openZ (:611): blinded Z has n + 3 coefficients (the SRS size)
        z = pyref.random_scalars(c, 1, 0x80)[0]
        bz = pyref.random_scalars(c, n + 3, 0x81)
        v = _eval(r, bz, z)
        q = _quotient(r, bz, v, z)
        assert len(q) == n + 2
        got = commit_checked(q, "open")
        want = oracle.batch_mul_base(CNAME, False, gen, enc([(_eval(r, bz, tau) - v) * pow(tau - z, -1, r) % r]))
        assert got == want, "open: quotient commitment != [(f(tau) - f(z)) / (tau - z)] G"
        # batchOpening (:757): six polynomials of different lengths, one gamma
        gamma = pyref.random_scalars(c, 1, 0x82)[0]
        lens = [n + 2, n + 3, n + 3, n + 3, n, n]
        polys = [pyref.random_scalars(c, m, 0x90 + i) for i, m in enumerate(lens)]
        claimed = [_eval(r, f, z) for f in polys]
        folded = [0] * max(lens)
        gi = 1
        for f in polys:
            for j, a in enumerate(f):
                folded[j] = (folded[j] + gi * a) % r
            gi = gi * gamma % r
        fz = 0
        for v_ in reversed(claimed):
            fz = (fz * gamma + v_) % r
        assert fz == _eval(r, folded, z)
        q = _quotient(r, folded, fz, z)
        got = commit_checked(q, "batch open")
        want = oracle.batch_mul_base(CNAME, False, gen, enc([(_eval(r, folded, tau) - fz) * pow(tau - z, -1, r) % r]))
        assert got == want, "batch open: quotient commitment mismatch"
        # computeNumerator (:949-967) on domain0, one polynomial through the GPU
        lag = enc(pyref.random_scalars(c, n, 0xA0))
        X = gm_ctx.copy_to_device(lag)
        gm_ctx.ntt(CNAME, X, n, True, False, False)  # ToCanonical: FFTInverse(DIF), Regular -> BitReverse
        canon_brev = X.to_host()
        assert canon_brev == oracle.fft(CNAME, lag, True, False, False)
        # the coefficients really are p's canonical ones, bit-reversed
        co = dec(canon_brev)
        nat = [co[pyref.bitrev(i, logn)] for i in range(n)]
        w0 = pyref.domain_generator(c, n)
        lv = dec(lag)
        for i in (0, 1, n - 1):
            assert _eval(r, nat, pow(w0, i, r)) == lv[i]
        # scale by the bit-reversed scaling vector (host, as prove.go:952-963), ToLagrange: FFT(DIT) -> Regular
        shift = pyref.random_scalars(c, 1, 0xA1)[0]
        sv = [pow(shift, pyref.bitrev(i, logn), r) for i in range(n)]
        scaled = enc([a * b % r for a, b in zip(co, sv)])
        X.write(scaled)
        gm_ctx.ntt(CNAME, X, n, False, True, False)
        assert X.to_host() == oracle.fft(CNAME, scaled, False, True, False)
        # :1016 / :1301: ToCanonical of a Lagrange BitReverse polynomial -> FFTInverse(DIT) -> Regular
        lag_br = enc(pyref.random_scalars(c, n, 0xA2))
        X.write(lag_br)
        gm_ctx.ntt(CNAME, X, n, True, True, False)
        assert X.to_host() == oracle.fft(CNAME, lag_br, True, True, False)
        X.free()
    finally:
        d_canon.free()
