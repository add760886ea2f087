"""Device-resident R1CS (gm_r1cs_*, csrc/r1cs.hip): solution.A / .B / .C
evaluated on the GPU from the wires -- <L_i, w>, <R_i, w>, <O_i, w>, the values
gnark's solver leaves in a, b, c (constraint/bn254/solver.go:540-620, terms
valued as computeTerm :144-173, constant terms included) -- and
gm_g16_prove_r1cs, the prover whose only per-proof host input is the wires.
Checked element for element against the host evaluation and, for proofs, byte
for byte against the oracle prover."""
import numpy as np
import pytest

import pyref
import r1cs as R
from test_groth16_gpu import TOXIC

pytestmark = pytest.mark.gpu


def _upload(gm_ctx, r1):
    import gnark_mi355x as gm
    return gm.R1CS.from_terms(gm_ctx, r1.curve, r1.nc, r1.nb_wires, r1.rowptr, r1.wires, r1.coeffs, r1.c.r)


def _eval(gm_ctx, handle, cname, W, nc):
    Wd = gm_ctx.copy_to_device(R.encode_vec(cname, W))
    bufs = [gm_ctx.malloc(32 * max(nc, 1)) for _ in range(3)]
    try:
        handle.eval(Wd, *bufs)
        return [b.to_host(32 * nc) for b in bufs]
    finally:
        for b in [Wd] + bufs:
            b.free()


@pytest.mark.parametrize("cname", ["bn254", "bls12377"])
def test_r1cs_eval_matches_solver_vectors(gm_ctx, cname):
    circuits = [R.cubic_circuit(cname), R.squaring_chain(300, cname, x=7)]
    r1, info, solve = R.commitment_chain(40, cname, 2)
    circuits.append((r1, solve(lambda i, h, p: sum(h) + 3 * sum(p) + i)))
    for r1, W in circuits:
        h = _upload(gm_ctx, r1)
        try:
            got = _eval(gm_ctx, h, cname, W, r1.nc)
        finally:
            h.free()
        a, b, cc = r1.solve_abc(W)
        assert got == [R.encode_vec(cname, v) for v in (a, b, cc)]


def test_r1cs_eval_constant_terms_and_coefficient_ids(gm_ctx):
    """Terms with the CoeffTable's fixed ids (0, 1, 2, -1, -2), circuit
    coefficients, constant terms (vid = GM_R1CS_CONST) and long rows."""
    import gnark_mi355x as gm
    cname = "bn254"
    c = pyref.CURVES[cname]
    r = c.r
    rng = np.random.default_rng(5)
    nw, nc = 50, 200
    W = [1] + [int(x) % r for x in rng.integers(1, 2 ** 62, nw - 1)]
    W[7] = r - 1
    table = [0, 1, 2, r - 1, r - 2] + [int(x) % r for x in rng.integers(3, 2 ** 60, 20)] + [r - 12345]
    rowptr, cid, vid = [], [], []
    exp = []
    for m in range(3):
        rp, ci, vi, ev = [0], [], [], []
        for i in range(nc):
            k = int(rng.integers(0, 4)) if i % 17 else 60  # empty rows and a few long ones
            acc = 0
            for _ in range(k):
                cc = int(rng.integers(0, len(table)))
                if rng.random() < 0.15:
                    vi.append(gm.R1CS_CONST)
                    acc += table[cc]
                else:
                    v = int(rng.integers(0, nw))
                    vi.append(v)
                    acc += table[cc] * W[v]
                ci.append(cc)
            rp.append(len(ci))
            ev.append(acc % r)
        rowptr.append(rp)
        cid.append(ci)
        vid.append(vi)
        exp.append(R.encode_vec(cname, ev))
    coeffs = R.encode_vec(cname, table)
    h = gm.R1CS(gm_ctx, cname, nc, nw, rowptr, cid, vid, coeffs)
    try:
        assert _eval(gm_ctx, h, cname, W, nc) == exp
    finally:
        h.free()
    # ids out of range are refused at upload
    bad = [list(x) for x in vid]
    bad[1][3] = nw
    with pytest.raises(gm.GmError, match="out of range"):
        gm.R1CS(gm_ctx, cname, nc, nw, rowptr, cid, bad, coeffs)
    badc = [list(x) for x in cid]
    badc[2][0] = len(table)
    with pytest.raises(gm.GmError, match="out of range"):
        gm.R1CS(gm_ctx, cname, nc, nw, rowptr, badc, vid, coeffs)


@pytest.mark.parametrize("cname,k,precompute", [("bn254", 1023, False), ("bn254", 4000, True),
                                                ("bls12377", 511, False)])
def test_groth16_prove_r1cs(gm_ctx, oracle, cname, k, precompute):
    """gm_g16_prove_r1cs (wires only over PCIe) == the oracle's proof."""
    import gnark_mi355x as gm
    c = pyref.CURVES[cname]
    r1, W = R.squaring_chain(k, cname, x=3)
    tox = R.encode_vec(cname, [t % c.r for t in TOXIC])
    pk = oracle.g16_setup(cname, r1, tox)
    a, b, cc = r1.solve_abc(W)
    enc = lambda v: R.encode_vec(cname, v)
    rb, sb = enc([0x77777]), enc([0x99999])
    exp = oracle.g16_prove(cname, pk, r1.nb_public, enc(W), enc(a), enc(b), enc(cc), rb, sb)
    dpk = gm.ProvingKey(gm_ctx, cname, pk, r1.domain_size, r1.nb_wires, r1.nb_public, precompute=precompute)
    h = _upload(gm_ctx, r1)
    try:
        assert dpk.prove_r1cs(h, enc(W), rb, sb) == exp
        assert dpk.prove_r1cs(h, enc(W), rb, sb) == exp  # resident state reused
    finally:
        h.free()
        dpk.free()
    assert oracle.g16_check(cname, r1, tox, enc(W), rb, sb, *exp) == 7


def test_groth16_prove_r1cs_bsb22(gm_ctx, oracle):
    """A commitment circuit (BSB22, prove.go:82-139) through the wires-only
    prover: the K filter from kWires and a, b, c from the resident R1CS."""
    import gnark_mi355x as gm
    cname = "bn254"
    c = pyref.CURVES[cname]
    r1, info, solve = R.commitment_chain(2000, cname, 2)
    tox = [t % c.r for t in TOXIC]
    sig = [0x31337, 0x4242]
    pk = oracle.g16_setup_bsb22(cname, r1, info, tox, sig)
    exp = oracle.g16_prove_bsb22(cname, pk, r1, info, solve, 0x1357, 0x2468)
    dpk = gm.ProvingKey(gm_ctx, cname, pk, r1.domain_size, r1.nb_wires, r1.nb_public)
    h = _upload(gm_ctx, r1)
    try:
        assert dpk.prove_r1cs(h, exp["Wb"], exp["rb"], exp["sb"]) == (exp["ar"], exp["bs"], exp["krs"])
        # a constraint system of another size is refused
        r2, _ = R.squaring_chain(10, cname)
        h2 = _upload(gm_ctx, r2)
        try:
            with pytest.raises(gm.GmError, match="does not match"):
                dpk.prove_r1cs(h2, exp["Wb"], exp["rb"], exp["sb"])
        finally:
            h2.free()
    finally:
        h.free()
        dpk.free()


@pytest.mark.parametrize("cname", ["bn254", "bls12377"])
def test_groth16_stage_prove_r1cs_wires_by_level(gm_ctx, oracle, cname):
    """gm_g16_stage_prove_r1cs: the wires handed over in pieces while Solve runs
    (GM_STAGE_WIRES ranges and indexed puts, as the wire-extended level hook of
    integration/go/solver_levelhook.diff delivers them), a, b, c evaluated from the
    resident R1CS -- the proof equals the oracle's; twice on one key (the stage
    buffers are reused), and a system of another size is refused."""
    import gnark_mi355x as gm
    c = pyref.CURVES[cname]
    r1, W = R.squaring_chain(1500 if cname == "bn254" else 400, cname, x=11)
    tox = R.encode_vec(cname, [t % c.r for t in TOXIC])
    pk = oracle.g16_setup(cname, r1, tox)
    a, b, cc = r1.solve_abc(W)
    enc = lambda v: R.encode_vec(cname, v)
    rb, sb = enc([0x5555]), enc([0x6666])
    exp = oracle.g16_prove(cname, pk, r1.nb_public, enc(W), enc(a), enc(b), enc(cc), rb, sb)
    dpk = gm.ProvingKey(gm_ctx, cname, pk, r1.domain_size, r1.nb_wires, r1.nb_public)
    h = _upload(gm_ctx, r1)
    Wb = enc(W)
    nw = r1.nb_wires
    try:
        for rep in range(2):
            st = dpk.stage(r1.nc)
            try:
                rng = np.random.default_rng(rep)
                st.put_range(st.WIRES, 0, Wb[:32 * r1.nb_public])  # the witness inputs
                rest = rng.permutation(np.arange(r1.nb_public, nw)) if rep else np.arange(r1.nb_public, nw)
                for lv in np.array_split(rest, 13):  # "levels" of solved wires
                    if rep:
                        st.put_indexed(st.WIRES, Wb, lv)
                    else:
                        st.put_range(st.WIRES, int(lv[0]), Wb[32 * int(lv[0]):32 * (int(lv[-1]) + 1)])
                assert st.prove_r1cs(h, rb, sb) == exp
            finally:
                st.free()
        r2, _ = R.squaring_chain(10, cname)
        h2 = _upload(gm_ctx, r2)
        st = dpk.stage(r1.nc)
        try:
            with pytest.raises(gm.GmError, match="does not match"):
                st.prove_r1cs(h2, rb, sb)
        finally:
            st.free()
            h2.free()
    finally:
        h.free()
        dpk.free()
