"""TEST ORACLE ONLY -- ctypes binding of the C++ CPU restatement (liboracle.so).

Imported by tests/, tests/golden/make_golden.py, __graft_entry__.smoke() and the
cpu_baseline leg of bench.py -- never by the product path.
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "_build", "liboracle.so")

CURVE_ID = {"bn254": 0, "bls12377": 1}
FP_BYTES = {"bn254": 32, "bls12377": 48}
FR_BYTES = 32

_lib = None

# Host threads the checker uses: the CPUs this process may run on, at most 16
# (a one-GPU box's CPU share; os.cpu_count() there reports the whole machine).
try:
    NTHREADS = max(1, min(16, len(os.sched_getaffinity(0))))
except AttributeError:  # pragma: no cover
    NTHREADS = max(1, min(16, os.cpu_count() or 1))


def build():
    subprocess.check_call(["make", "-s", "-C", HERE])


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            build()
        L = ctypes.CDLL(LIB_PATH)
        vp, sz, i = ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int
        L.o_msm.argtypes = [i, i, vp, vp, sz, i, i, vp]
        L.o_fft.argtypes = [i, vp, sz, i, i, i, i]
        L.o_compute_h.argtypes = [i, vp, vp, vp, sz, sz, i, vp]
        L.o_batch_mul_base.argtypes = [i, i, vp, vp, sz, i, vp]
        L.o_generator.argtypes = [i, i]
        L.o_generator.restype = ctypes.POINTER(ctypes.c_uint8)
        L.o_g16_setup.argtypes = [i, sz, sz, sz, vp, vp, vp, vp, vp, vp, vp, vp, i]
        L.o_g16_prove.argtypes = [i, vp, vp, vp, vp, sz, vp, vp, vp, vp, sz, vp, vp, i, vp, vp, vp]
        L.o_g16_check.argtypes = [i, sz, sz, sz, vp, vp, vp, vp, vp, vp, vp, vp, vp, vp]
        L.o_g16_check_mask.argtypes = [i, sz, sz, sz, vp, vp, vp, vp, vp, vp, vp, vp, vp, vp, vp]
        _lib = L
    return _lib


def _ptr(a: np.ndarray):
    return a.ctypes.data_as(ctypes.c_void_p)


def _u8(b) -> np.ndarray:
    if isinstance(b, np.ndarray):
        return np.ascontiguousarray(b.view(np.uint8).reshape(-1))
    return np.frombuffer(bytes(b), dtype=np.uint8).copy()


def point_bytes(curve: str, g2: bool) -> int:
    return FP_BYTES[curve] * (4 if g2 else 2)


def msm(curve: str, g2: bool, scalars, points, nthreads: int = 0, naive: bool = False) -> bytes:
    nthreads = nthreads or NTHREADS
    s = _u8(scalars)
    p = _u8(points)
    n = s.size // FR_BYTES
    assert p.size == n * point_bytes(curve, g2)
    out = np.zeros(point_bytes(curve, g2), dtype=np.uint8)
    rc = lib().o_msm(CURVE_ID[curve], int(g2), _ptr(s), _ptr(p), n, nthreads, int(naive), _ptr(out))
    assert rc == 0
    return out.tobytes()


def fft(curve: str, data, inverse: bool, dit: bool, coset: bool, nthreads: int = 0) -> bytes:
    nthreads = nthreads or NTHREADS
    a = _u8(data).copy()
    n = a.size // FR_BYTES
    rc = lib().o_fft(CURVE_ID[curve], _ptr(a), n, int(inverse), int(dit), int(coset), nthreads)
    assert rc == 0, rc
    return a.tobytes()


def compute_h(curve: str, a, b, c, n: int, nthreads: int = 0) -> bytes:
    nthreads = nthreads or NTHREADS
    A, B, C = _u8(a), _u8(b), _u8(c)
    ln = A.size // FR_BYTES
    out = np.zeros(n * FR_BYTES, dtype=np.uint8)
    rc = lib().o_compute_h(CURVE_ID[curve], _ptr(A), _ptr(B), _ptr(C), ln, n, nthreads, _ptr(out))
    assert rc == 0
    return out.tobytes()


def generator(curve: str, g2: bool) -> bytes:
    p = lib().o_generator(CURVE_ID[curve], int(g2))
    return bytes(p[: point_bytes(curve, g2)])


def batch_mul_base(curve: str, g2: bool, base: bytes, scalars, nthreads: int = 0) -> bytes:
    nthreads = nthreads or NTHREADS
    s = _u8(scalars)
    n = s.size // FR_BYTES
    b = _u8(base)
    out = np.zeros(n * point_bytes(curve, g2), dtype=np.uint8)
    rc = lib().o_batch_mul_base(CURVE_ID[curve], int(g2), _ptr(b), _ptr(s), n, nthreads, _ptr(out))
    assert rc == 0
    return out.tobytes()


# ---------------------------------------------------------------------------
# Groth16 helpers (R1CS in CSR form, see tests/r1cs.py)
# ---------------------------------------------------------------------------
def _ptr_array(arrs):
    keep = [np.ascontiguousarray(a) for a in arrs]
    ptrs = (ctypes.c_void_p * len(keep))(*[a.ctypes.data for a in keep])
    return ptrs, keep


def g16_setup(curve: str, r1cs, toxic: bytes, nthreads: int = 0):
    """Returns a dict with the proving-key arrays (gnark layout bytes)."""
    nthreads = nthreads or NTHREADS
    fpb = FP_BYTES[curve]
    g1b, g2b = 2 * fpb, 4 * fpb
    n = r1cs.domain_size
    sizes = np.array([n, r1cs.nb_wires, r1cs.nbA, r1cs.nbB, r1cs.nb_wires - r1cs.nb_public],
                     dtype=np.uint64)
    pk = {
        "g1_alpha": np.zeros(g1b, np.uint8), "g1_beta": np.zeros(g1b, np.uint8),
        "g1_delta": np.zeros(g1b, np.uint8),
        "g1_A": np.zeros(g1b * r1cs.nbA, np.uint8), "g1_B": np.zeros(g1b * r1cs.nbB, np.uint8),
        "g1_Z": np.zeros(g1b * (n - 1), np.uint8),
        "g1_K": np.zeros(g1b * (r1cs.nb_wires - r1cs.nb_public), np.uint8),
        "g2_beta": np.zeros(g2b, np.uint8), "g2_delta": np.zeros(g2b, np.uint8),
        "g2_B": np.zeros(g2b * r1cs.nbB, np.uint8),
        "infA": np.zeros(r1cs.nb_wires, np.uint8), "infB": np.zeros(r1cs.nb_wires, np.uint8),
    }
    rp, k1 = _ptr_array(r1cs.rowptr)
    wi, k2 = _ptr_array(r1cs.wires)
    co, k3 = _ptr_array(r1cs.coeffs)
    g1, k4 = _ptr_array([pk[k] for k in ["g1_alpha", "g1_beta", "g1_delta", "g1_A", "g1_B", "g1_Z", "g1_K"]])
    g2, k5 = _ptr_array([pk[k] for k in ["g2_beta", "g2_delta", "g2_B"]])
    inf, k6 = _ptr_array([pk["infA"], pk["infB"]])
    tox = _u8(toxic)
    rc = lib().o_g16_setup(CURVE_ID[curve], r1cs.nc, r1cs.nb_wires, r1cs.nb_public, rp, wi, co,
                           _ptr(tox), _ptr(sizes), g1, g2, inf, nthreads)
    assert rc == 0, rc
    pk["sizes"] = sizes
    return pk


def g16_prove(curve: str, pk, nb_public: int, wires, a, b, c, r: bytes, s: bytes, nthreads: int = 0):
    nthreads = nthreads or NTHREADS
    fpb = FP_BYTES[curve]
    g1, k4 = _ptr_array([pk[k] for k in ["g1_alpha", "g1_beta", "g1_delta", "g1_A", "g1_B", "g1_Z", "g1_K"]])
    g2, k5 = _ptr_array([pk[k] for k in ["g2_beta", "g2_delta", "g2_B"]])
    inf, k6 = _ptr_array([pk["infA"], pk["infB"]])
    W, A, B, C = _u8(wires), _u8(a), _u8(b), _u8(c)
    R, S = _u8(r), _u8(s)
    ar = np.zeros(2 * fpb, np.uint8)
    krs = np.zeros(2 * fpb, np.uint8)
    bs = np.zeros(4 * fpb, np.uint8)
    rc = lib().o_g16_prove(CURVE_ID[curve], _ptr(pk["sizes"]), g1, g2, inf, nb_public, _ptr(W),
                           _ptr(A), _ptr(B), _ptr(C), A.size // 32, _ptr(R), _ptr(S), nthreads,
                           _ptr(ar), _ptr(bs), _ptr(krs))
    assert rc == 0, rc
    return ar.tobytes(), bs.tobytes(), krs.tobytes()


def g16_check(curve: str, r1cs, toxic: bytes, wires, r: bytes, s: bytes, ar: bytes, bs: bytes,
              krs: bytes, vk_mask=None) -> int:
    """7 = (Ar, Bs, Krs) satisfy the verification equation in the exponent.
    vk_mask: per-wire verifier-side flags (BSB22: public + commitment +
    private committed wires); default: the public wires."""
    rp, k1 = _ptr_array(r1cs.rowptr)
    wi, k2 = _ptr_array(r1cs.wires)
    co, k3 = _ptr_array(r1cs.coeffs)
    arrs = [_u8(x) for x in (toxic, wires, r, s, ar, bs, krs)]
    if vk_mask is None:
        return lib().o_g16_check(CURVE_ID[curve], r1cs.nc, r1cs.nb_wires, r1cs.nb_public, rp, wi, co,
                                 *[_ptr(x) for x in arrs])
    m = np.asarray(vk_mask, dtype=np.uint8)
    assert m.size == r1cs.nb_wires
    return lib().o_g16_check_mask(CURVE_ID[curve], r1cs.nc, r1cs.nb_wires, r1cs.nb_public, rp, wi, co,
                                  *[_ptr(x) for x in arrs], _ptr(m))


# ----------------------------------------------------------------------------
# BSB22 commitments (prove.go:82-139, setup.go:143-196 + 278-305): the Groth16
# restatement above plus the commitment side path.  `info` is the circuit's
# constraint.Groth16Commitments: dicts with public_and_commitment_committed,
# nb_public_committed, private_committed (sorted wire ids), commitment_index.
# ----------------------------------------------------------------------------
def bsb22_k_wires(info, nb_public: int, nb_wires: int):
    """The wires of pk.G1.K: private wires minus private-committed and
    commitment wires (setup.go:164-195; the prover's filterHeap, prove.go:243-245)."""
    drop = set(w for ci in info for w in ci["private_committed"]) | set(ci["commitment_index"] for ci in info)
    return [w for w in range(nb_public, nb_wires) if w not in drop]


def bsb22_vk_mask(info, nb_public: int, nb_wires: int):
    """Wires on the verifier's side: public, commitment (vkK, setup.go:184-186)
    and private committed (inside the commitments D_i, verify.go:121-123)."""
    side = set(range(nb_public)) | set(ci["commitment_index"] for ci in info)
    side |= set(w for ci in info for w in ci["private_committed"])
    return [1 if w in side else 0 for w in range(nb_wires)]


def g16_setup_bsb22(curve: str, r1cs, info, toxic_vals, sigmas, nthreads: int = 0):
    """Setup with commitments.  The C++ setup gives K_w = (beta A_w + alpha B_w +
    C_w) / delta [G1] for every private wire; pk.G1.K keeps the bsb22_k_wires
    ones, and commitment i's Pedersen basis (setup.go:188, :278-305) is the
    committed wires' (beta A + alpha B + C) / gamma [G1] = (delta / gamma) K_w,
    BasisExpSigma = sigma_i Basis (pedersen.Setup with sigma_i)."""
    import pyref
    c = pyref.CURVES[curve]
    toxic = b"".join(pyref.encode_fr(c, t % c.r) for t in toxic_vals)
    pk = g16_setup(curve, r1cs, toxic, nthreads)
    g1b = 2 * FP_BYTES[curve]
    nbk_full = r1cs.nb_wires - r1cs.nb_public
    Kfull = np.frombuffer(pk["g1_K"], np.uint8).reshape(nbk_full, g1b)
    kw = bsb22_k_wires(info, r1cs.nb_public, r1cs.nb_wires)
    pk["g1_K_full"] = pk["g1_K"]
    pk["g1_K"] = Kfull[[w - r1cs.nb_public for w in kw]].reshape(-1).copy()
    pk["k_wires"] = kw
    G = pyref.Group(c, False)
    _, _, _, gamma, delta = (t % c.r for t in toxic_vals)
    dg = delta * pow(gamma, -1, c.r) % c.r
    pk["ck"] = []
    for ci, sg in zip(info, sigmas):
        basis = [G.mul(pyref.decode_point(c, Kfull[w - r1cs.nb_public].tobytes(), False), dg)
                 for w in ci["private_committed"]]
        pk["ck"].append({
            "basis": b"".join(pyref.encode_point(c, P, False) for P in basis),
            "basis_sigma": b"".join(pyref.encode_point(c, G.mul(P, sg % c.r), False) for P in basis),
        })
    pk["sizes"][4] = len(kw)
    pk["toxic"] = toxic
    return pk


def g16_prove_bsb22(curve: str, pk, r1cs, info, solve, r: int, s: int, nthreads: int = 0):
    """prove.go:62-313 with commitments.  solve(hint) returns the witness; hint
    is the overridden Bsb22CommitmentComputePlaceholder (prove.go:83-108).
    Returns dict(W, a, b, c, ar, bs, krs, commitments, pok) (byte strings in
    gnark layout; W, a, b, c Montgomery)."""
    import pyref
    c = pyref.CURVES[curve]
    enc = lambda vals: b"".join(pyref.encode_fr(c, v % c.r) for v in vals)
    commitments, committed = [None] * len(info), [None] * len(info)

    def hint(i, hashed, priv):
        committed[i] = [v % c.r for v in priv]
        D = msm(curve, False, enc(committed[i]), pk["ck"][i]["basis"], nthreads)
        commitments[i] = D
        return pyref.bsb22_commitment_value(c, pyref.decode_point(c, D, False), hashed)

    W = solve(hint)
    a, b, cc = r1cs.solve_abc(W)
    poks = [pyref.decode_point(c, msm(curve, False, enc(committed[i]), pk["ck"][i]["basis_sigma"], nthreads), False)
            for i in range(len(info))]
    chal = pyref.pok_challenge(c, [W[ci["commitment_index"]] for ci in info])
    pok = pyref.encode_point(c, pyref.fold_points(c, poks, chal), False)
    # Groth16 core with the K filter of prove.go:243-245: the dropped wires'
    # K points set to infinity in the full key
    g1b = 2 * FP_BYTES[curve]
    nbk_full = r1cs.nb_wires - r1cs.nb_public
    Kz = np.frombuffer(pk["g1_K_full"], np.uint8).reshape(nbk_full, g1b).copy()
    keep = np.zeros(nbk_full, bool)
    keep[[w - r1cs.nb_public for w in pk["k_wires"]]] = True
    Kz[~keep] = 0
    full = dict(pk)
    full["g1_K"] = Kz.reshape(-1)
    full["sizes"] = pk["sizes"].copy()
    full["sizes"][4] = nbk_full
    ar, bs, krs = g16_prove(curve, full, r1cs.nb_public, enc(W), enc(a), enc(b), enc(cc), enc([r]), enc([s]),
                            nthreads)
    return {"W": W, "Wb": enc(W), "a": enc(a), "b": enc(b), "c": enc(cc), "ar": ar, "bs": bs, "krs": krs,
            "commitments": commitments, "pok": pok, "rb": enc([r]), "sb": enc([s])}


def bsb22_check(curve: str, r1cs, pk, info, proof, sigmas) -> bool:
    """verify.go:49-150 in the exponent: the Groth16 equation with the BSB22
    verifier-side wires, plus pedersen.BatchVerifyMultiVk's statement
    pok = sum_i chal^i sigma_i D_i (the pairing form of it holds iff this does)."""
    import pyref
    c = pyref.CURVES[curve]
    ok = g16_check(curve, r1cs, pk["toxic"], proof["Wb"], proof["rb"], proof["sb"], proof["ar"], proof["bs"],
                   proof["krs"], bsb22_vk_mask(info, r1cs.nb_public, r1cs.nb_wires)) == 7
    G = pyref.Group(c, False)
    chal = pyref.pok_challenge(c, [proof["W"][ci["commitment_index"]] for ci in info])
    want, e = None, 1
    for D, sg in zip(proof["commitments"], sigmas):
        want = G.add(want, G.mul(pyref.decode_point(c, D, False), e * sg % c.r))
        e = e * chal % c.r
    return ok and pyref.encode_point(c, want, False) == proof["pok"]
