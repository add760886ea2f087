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
              krs: bytes) -> int:
    rp, k1 = _ptr_array(r1cs.rowptr)
    wi, k2 = _ptr_array(r1cs.wires)
    co, k3 = _ptr_array(r1cs.coeffs)
    arrs = [_u8(x) for x in (toxic, wires, r, s, ar, bs, krs)]
    return lib().o_g16_check(CURVE_ID[curve], r1cs.nc, r1cs.nb_wires, r1cs.nb_public, rp, wi, co,
                             *[_ptr(x) for x in arrs])
