"""Python binding of libgnark_mi355x.so (ctypes) -- host plumbing for tests and
bench.py.  The product is the C-ABI in include/gnark_mi355x.h; this module only
mirrors it, keeping iciclegnark's operation names
(backend/groth16/bn254/icicle/icicle.go call sites) so tests read like the
reference's own flow:

    CopyToDevice          -> copy_to_device            (icicle.go:44,47,65,245,269,352,478-480)
    CopyPointsToDevice    -> copy_points_to_device     (icicle.go:90,95,109,114)
    CopyG2PointsToDevice  -> copy_points_to_device(g2=True)  (icicle.go:125)
    GenerateTwiddleFactors-> generate_twiddle_factors  (icicle.go:68,73)
    INttOnDevice          -> intt_on_device            (icicle.go:489,502)
    NttOnDevice           -> ntt_on_device             (icicle.go:490)
    PolyOps               -> poly_ops                  (icicle.go:500)
    ReverseScalars        -> reverse_scalars           (icicle.go:510)
    MsmOnDevice           -> msm_on_device             (icicle.go:302,315,332,355)
    MsmG2OnDevice         -> msm_g2_on_device          (icicle.go:382)
    FreeDevicePointer     -> free_device_pointer       (icicle.go:356,416-418,492,505-507)
    icicle_bn254.Prove    -> ProvingKey.prove          (icicle.go:133-422)

There is NO fallback: if the shared library is missing or no GPU is visible the
calls raise.
"""
from __future__ import annotations

import ctypes
import os
import struct

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
# GNARK_MI355X_LIB: an alternative build of the same library (same-box A/B runs)
LIB_PATH = os.environ.get("GNARK_MI355X_LIB") or os.path.join(HERE, "libgnark_mi355x.so")

BN254, BLS12_377 = 0, 1
CURVES = {"bn254": BN254, "bls12377": BLS12_377}
FP_BYTES = {BN254: 32, BLS12_377: 48}
FR_BYTES = 32

# exported symbols (include/gnark_mi355x.h) -- checked by tests/test_capi_symbols.py
SYMBOLS = [
    "gm_last_error", "gm_version", "gm_init", "gm_destroy", "gm_synchronize", "gm_trim",
    "gm_profile_enable", "gm_profile_reset", "gm_profile_get", "gm_profile_dump",
    "gm_set_msm_window", "gm_set_msm_glv", "gm_malloc", "gm_free", "gm_copy_to_device", "gm_memcpy_h2d",
    "gm_memcpy_d2h", "gm_memcpy_d2d", "gm_copy_points_to_device", "gm_msm", "gm_msm_host_scalars", "gm_points_upload", "gm_msm_prepared", "gm_precompute_layout", "gm_points_upload_precomputed",
    "gm_msm_precomputed", "gm_kzg_commit", "gm_ntt",
    "gm_poly_ops", "gm_reverse_scalars", "gm_groth16_compute_h", "gm_g16_pk_upload", "gm_g16_pk_upload_ex", "gm_g16_pk_upload_shard",
    "gm_g16_partial_bytes", "gm_g16_prove_partial", "gm_g16_finish",
    "gm_g16_pk_free", "gm_g16_pk_precomputed", "gm_g16_prove", "gm_g16_prove_device", "gm_jac_add", "gm_jac_to_affine",
    "gm_batch_mul_base", "gm_random_scalars", "gm_generator", "gm_icicle_generate_twiddles", "gm_icicle_intt_on_device", "gm_icicle_ntt_on_device",
    "gm_icicle_poly_ops", "gm_device_count", "gm_multi_init", "gm_multi_destroy", "gm_multi_size",
    "gm_multi_context", "gm_g16_pk_upload_multi", "gm_g16_pk_free_multi", "gm_g16_prove_multi",
    "gm_g16_pk_upload_dump", "gm_g16_pk_upload_dump_shard", "gm_g16_pk_save_cache", "gm_g16_pk_load_cache",
    "gm_g16_stage_begin", "gm_g16_stage_put_range", "gm_g16_stage_put_indexed", "gm_g16_stage_prove",
    "gm_g16_stage_free", "gm_msm_async", "gm_msm_wait", "gm_r1cs_upload", "gm_r1cs_free", "gm_r1cs_eval",
    "gm_g16_prove_r1cs", "gm_g16_stage_prove_r1cs",
]
# test-only library (include/gnark_mi355x_testhooks.h, libgnark_mi355x_testhooks.so)
TEST_SYMBOLS = ["gm_test_field_op", "gm_test_point_op", "gm_test_stage_replay_chain"]
TESTHOOKS_PATH = os.path.join(os.path.dirname(LIB_PATH), "libgnark_mi355x_testhooks.so")


class GmError(RuntimeError):
    pass


_lib = None
_testhooks = None


def load_testhooks(path: str = None):
    """The test-only element-wise hooks (parity tests of the field / curve layer);
    loads the product library first (the hooks link against it)."""
    global _testhooks
    if _testhooks is not None:
        return _testhooks
    load_library()
    path = path or TESTHOOKS_PATH
    if not os.path.exists(path):
        raise GmError(f"{path} not built -- run `make -C gnark-icicle_amd`")
    T = ctypes.CDLL(path)
    vp, sz, i = ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int
    T.gm_test_field_op.argtypes = [vp, i, i, i, vp, vp, vp, sz]
    T.gm_test_point_op.argtypes = [vp, i, i, i, vp, vp, vp, sz]
    T.gm_test_stage_replay_chain.argtypes = [vp, vp, sz, vp, vp, vp, sz, i, i, sz, ctypes.POINTER(ctypes.c_double)]
    _testhooks = T
    return T


def load_library(path: str = LIB_PATH):
    """Loads the C-ABI library (raises if it has not been built)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(path):
        raise GmError(f"{path} not built -- run `make -C gnark-icicle_amd` (or __graft_entry__.build())")
    L = ctypes.CDLL(path)
    vp, sz, i, u64 = ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int, ctypes.c_uint64
    pvp = ctypes.POINTER(ctypes.c_void_p)
    L.gm_last_error.restype = ctypes.c_char_p
    L.gm_init.argtypes = [i, pvp]
    L.gm_destroy.argtypes = [vp]
    L.gm_synchronize.argtypes = [vp]
    L.gm_trim.argtypes = [vp]
    L.gm_profile_enable.argtypes = [vp, i]
    L.gm_profile_reset.argtypes = [vp]
    L.gm_profile_get.argtypes = [vp, ctypes.c_char_p, ctypes.POINTER(ctypes.c_double), ctypes.POINTER(u64)]
    L.gm_profile_dump.argtypes = [vp, ctypes.c_char_p, sz]
    L.gm_set_msm_window.argtypes = [vp, i]
    L.gm_set_msm_glv.argtypes = [vp, i]
    L.gm_malloc.argtypes = [vp, sz, pvp]
    L.gm_free.argtypes = [vp, vp]
    L.gm_copy_to_device.argtypes = [vp, vp, sz, pvp]
    L.gm_memcpy_h2d.argtypes = [vp, vp, vp, sz]
    L.gm_memcpy_d2h.argtypes = [vp, vp, vp, sz]
    L.gm_memcpy_d2d.argtypes = [vp, vp, vp, sz]
    L.gm_copy_points_to_device.argtypes = [vp, i, i, vp, sz, pvp]
    L.gm_msm.argtypes = [vp, i, i, vp, vp, sz, vp, vp]
    L.gm_msm_host_scalars.argtypes = [vp, i, i, vp, vp, sz, vp, vp]
    L.gm_points_upload.argtypes = [vp, i, i, vp, sz, pvp]
    L.gm_msm_prepared.argtypes = [vp, i, i, vp, vp, sz, vp, vp]
    L.gm_precompute_layout.argtypes = [i, sz, i, ctypes.POINTER(i), ctypes.POINTER(i)]
    L.gm_points_upload_precomputed.argtypes = [vp, i, i, vp, sz, i, pvp]
    L.gm_msm_precomputed.argtypes = [vp, i, i, vp, vp, sz, i, sz, vp, vp]
    L.gm_kzg_commit.argtypes = [vp, i, vp, sz, vp, sz, vp]
    L.gm_ntt.argtypes = [vp, i, vp, sz, i, i, i]
    L.gm_poly_ops.argtypes = [vp, i, vp, vp, vp, sz, vp]
    L.gm_reverse_scalars.argtypes = [vp, i, vp, sz]
    L.gm_groth16_compute_h.argtypes = [vp, i, vp, vp, vp, sz, sz]
    L.gm_g16_pk_upload.argtypes = [vp, i, vp, pvp]
    L.gm_g16_pk_upload_ex.argtypes = [vp, i, vp, ctypes.c_uint, pvp]
    L.gm_g16_pk_upload_shard.argtypes = [vp, i, vp, ctypes.c_uint, i, i, pvp]
    L.gm_g16_partial_bytes.argtypes = [i, ctypes.POINTER(sz)]
    L.gm_g16_prove_partial.argtypes = [vp, vp, vp, vp, vp, vp, sz, vp]
    L.gm_g16_finish.argtypes = [i, vp, vp, vp, vp, vp, vp, vp]
    L.gm_g16_pk_free.argtypes = [vp, vp]
    L.gm_g16_pk_precomputed.argtypes = [vp, ctypes.POINTER(ctypes.c_int)]
    L.gm_g16_prove.argtypes = [vp, vp, vp, vp, vp, vp, sz, vp, vp, vp, vp, vp]
    L.gm_g16_prove_device.argtypes = [vp, vp, vp, vp, vp, vp, sz, vp, vp, vp, vp, vp]
    L.gm_r1cs_upload.argtypes = [vp, i, sz, sz, vp, vp, vp, vp, sz, vp]
    L.gm_r1cs_free.argtypes = [vp, vp]
    L.gm_r1cs_eval.argtypes = [vp, vp, vp, vp, vp, vp]
    L.gm_g16_prove_r1cs.argtypes = [vp, vp, vp, vp, vp, vp, vp, vp, vp]
    L.gm_jac_add.argtypes = [i, i, vp, vp, vp]
    L.gm_jac_to_affine.argtypes = [i, i, vp, vp]
    L.gm_batch_mul_base.argtypes = [vp, i, i, vp, vp, sz, vp]
    L.gm_random_scalars.argtypes = [vp, i, u64, sz, vp]
    L.gm_generator.argtypes = [i, i, vp]
    L.gm_icicle_generate_twiddles.argtypes = [vp, i, sz, i, pvp]
    L.gm_icicle_intt_on_device.argtypes = [vp, i, vp, sz, i, pvp]
    L.gm_icicle_ntt_on_device.argtypes = [vp, i, vp, vp, sz, i]
    L.gm_icicle_poly_ops.argtypes = [vp, i, vp, vp, vp, vp, sz]
    L.gm_device_count.argtypes = [ctypes.POINTER(i)]
    L.gm_multi_init.argtypes = [ctypes.POINTER(i), i, pvp]
    L.gm_multi_destroy.argtypes = [vp]
    L.gm_multi_size.argtypes = [vp, ctypes.POINTER(i)]
    L.gm_multi_context.argtypes = [vp, i, pvp]
    L.gm_g16_pk_upload_multi.argtypes = [vp, i, vp, ctypes.c_uint, pvp]
    L.gm_g16_pk_free_multi.argtypes = [vp, vp]
    L.gm_g16_prove_multi.argtypes = [vp, vp, vp, vp, vp, vp, sz, vp, vp, vp, vp, vp]
    L.gm_g16_pk_upload_dump.argtypes = [vp, i, vp, i, u64, ctypes.c_uint, ctypes.POINTER(u64), pvp]
    L.gm_g16_pk_upload_dump_shard.argtypes = [vp, i, vp, i, u64, ctypes.c_uint, i, i, ctypes.POINTER(u64), pvp]
    L.gm_g16_pk_save_cache.argtypes = [vp, vp, i]
    L.gm_g16_pk_load_cache.argtypes = [vp, i, pvp]
    L.gm_g16_stage_begin.argtypes = [vp, vp, sz, pvp]
    L.gm_g16_stage_put_range.argtypes = [vp, i, sz, sz, vp]
    L.gm_g16_stage_put_indexed.argtypes = [vp, i, vp, vp, sz]
    L.gm_g16_stage_prove.argtypes = [vp, vp, vp, vp, vp, vp]
    L.gm_g16_stage_free.argtypes = [vp]
    L.gm_g16_stage_prove_r1cs.argtypes = [vp, vp, vp, vp, vp, vp, vp]
    L.gm_msm_async.argtypes = [vp, i, i, vp, vp, sz, pvp]
    L.gm_msm_wait.argtypes = [vp, vp, vp]
    _lib = L
    return L


def _check(rc: int):
    if rc != 0:
        raise GmError(f"gnark_mi355x error {rc}: {load_library().gm_last_error().decode()}")


def _buf(b) -> np.ndarray:
    if isinstance(b, np.ndarray):
        return np.ascontiguousarray(b).view(np.uint8).reshape(-1)
    return np.frombuffer(bytes(b), dtype=np.uint8)


def _p(a: np.ndarray):
    return a.ctypes.data_as(ctypes.c_void_p)


def curve_id(curve) -> int:
    return CURVES[curve] if isinstance(curve, str) else int(curve)


def point_bytes(curve, g2: bool) -> int:
    return FP_BYTES[curve_id(curve)] * (4 if g2 else 2)


def jac_bytes(curve, g2: bool) -> int:
    return FP_BYTES[curve_id(curve)] * (6 if g2 else 3)


def generator(curve, g2: bool = False) -> bytes:
    out = np.zeros(point_bytes(curve, g2), np.uint8)
    _check(load_library().gm_generator(curve_id(curve), int(g2), _p(out)))
    return out.tobytes()


def jac_add(curve, g2: bool, p: bytes, q: bytes) -> bytes:
    out = np.zeros(jac_bytes(curve, g2), np.uint8)
    a, b = _buf(p), _buf(q)
    _check(load_library().gm_jac_add(curve_id(curve), int(g2), _p(a), _p(b), _p(out)))
    return out.tobytes()


def jac_to_affine(curve, g2: bool, p: bytes) -> bytes:
    out = np.zeros(point_bytes(curve, g2), np.uint8)
    a = _buf(p)
    _check(load_library().gm_jac_to_affine(curve_id(curve), int(g2), _p(a), _p(out)))
    return out.tobytes()


class DeviceBuffer:
    """A device allocation owned by a Context (OnDeviceData{P, Size}, icicle.go:228)."""

    def __init__(self, ctx: "Context", ptr: int, nbytes: int):
        self.ctx, self.ptr, self.nbytes = ctx, ptr, nbytes

    def to_host(self, nbytes: int | None = None) -> bytes:
        n = self.nbytes if nbytes is None else nbytes
        out = np.zeros(n, np.uint8)
        _check(load_library().gm_memcpy_d2h(self.ctx.handle, _p(out), self.ptr, n))
        return out.tobytes()

    def write(self, data, offset: int = 0):
        a = _buf(data)
        _check(load_library().gm_memcpy_h2d(self.ctx.handle, self.ptr + offset, _p(a), a.size))

    def copy_from(self, src: "DeviceBuffer", nbytes: int | None = None):
        n = min(self.nbytes, src.nbytes) if nbytes is None else nbytes
        _check(load_library().gm_memcpy_d2d(self.ctx.handle, self.ptr, src.ptr, n))

    def free(self):
        if self.ptr:
            _check(load_library().gm_free(self.ctx.handle, self.ptr))
            self.ptr = 0


class Context:
    """One HIP device + stream (gm_ctx)."""

    def __init__(self, device: int = 0):
        L = load_library()
        h = ctypes.c_void_p()
        _check(L.gm_init(device, ctypes.byref(h)))
        self.handle = h
        self.device = device

    def trim(self):
        """gm_trim: release the memory the context keeps between calls."""
        _check(load_library().gm_trim(self.handle))

    def close(self):
        if self.handle:
            load_library().gm_destroy(self.handle)
            self.handle = None

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    # ---- memory ----------------------------------------------------------
    def malloc(self, nbytes: int) -> DeviceBuffer:
        p = ctypes.c_void_p()
        _check(load_library().gm_malloc(self.handle, nbytes, ctypes.byref(p)))
        return DeviceBuffer(self, p.value, nbytes)

    def copy_to_device(self, data) -> DeviceBuffer:
        a = _buf(data)
        p = ctypes.c_void_p()
        _check(load_library().gm_copy_to_device(self.handle, _p(a), a.size, ctypes.byref(p)))
        return DeviceBuffer(self, p.value, a.size)

    def copy_points_to_device(self, curve, points, g2: bool = False) -> DeviceBuffer:
        a = _buf(points)
        n = a.size // point_bytes(curve, g2)
        p = ctypes.c_void_p()
        _check(load_library().gm_copy_points_to_device(self.handle, curve_id(curve), int(g2), _p(a), n,
                                                       ctypes.byref(p)))
        return DeviceBuffer(self, p.value, a.size)

    def free_device_pointer(self, buf: DeviceBuffer):
        buf.free()

    def synchronize(self):
        _check(load_library().gm_synchronize(self.handle))

    # ---- profiling ---------------------------------------------------------
    def profile(self, on: bool = True):
        _check(load_library().gm_profile_enable(self.handle, int(on)))

    def profile_reset(self):
        _check(load_library().gm_profile_reset(self.handle))

    def profile_stats(self) -> dict:
        buf = ctypes.create_string_buffer(1 << 16)
        _check(load_library().gm_profile_dump(self.handle, buf, len(buf)))
        out = {}
        for line in buf.value.decode().splitlines():
            name, ms, cnt = line.split()
            out[name] = (float(ms), int(cnt))
        return out

    def set_msm_window(self, c: int):
        _check(load_library().gm_set_msm_window(self.handle, c))

    def set_msm_glv(self, mode: int):
        """GLV split of plain MSMs: 1 on, 0 off, -1 the size rule (on up to 2^21 points)."""
        _check(load_library().gm_set_msm_glv(self.handle, mode))

    # ---- MSM -----------------------------------------------------------------
    def msm(self, curve, scalars: DeviceBuffer, points: DeviceBuffer, n: int, g2: bool = False):
        """Returns (jacobian_bytes, affine_bytes) in gnark layout."""
        jac = np.zeros(jac_bytes(curve, g2), np.uint8)
        aff = np.zeros(point_bytes(curve, g2), np.uint8)
        sp = scalars.ptr if isinstance(scalars, DeviceBuffer) else scalars
        pp = points.ptr if isinstance(points, DeviceBuffer) else points
        _check(load_library().gm_msm(self.handle, curve_id(curve), int(g2), sp, pp, n, _p(jac), _p(aff)))
        return jac.tobytes(), aff.tobytes()

    def msm_async(self, curve, scalars: DeviceBuffer, points: DeviceBuffer, n: int, g2: bool = False):
        """Queues an MSM (gm_msm_async); .wait() returns (jacobian_bytes, affine_bytes).
        At most three in flight per context, waited in issue order."""
        h = ctypes.c_void_p()
        sp = scalars.ptr if isinstance(scalars, DeviceBuffer) else scalars
        pp = points.ptr if isinstance(points, DeviceBuffer) else points
        _check(load_library().gm_msm_async(self.handle, curve_id(curve), int(g2), sp, pp, n, ctypes.byref(h)))
        return PendingMsm(h, curve, g2)

    def points_upload(self, curve, points, g2: bool = False) -> DeviceBuffer:
        """Device-resident point set in the MSM's internal layout (pk arrays, SRS)."""
        a = _buf(points)
        n = a.size // point_bytes(curve, g2)
        p = ctypes.c_void_p()
        _check(load_library().gm_points_upload(self.handle, curve_id(curve), int(g2), _p(a), n, ctypes.byref(p)))
        buf = DeviceBuffer(self, p.value, a.size)
        buf.count = n
        return buf

    def msm_prepared(self, curve, scalars: DeviceBuffer, prepared: DeviceBuffer, n: int, g2: bool = False):
        jac = np.zeros(jac_bytes(curve, g2), np.uint8)
        aff = np.zeros(point_bytes(curve, g2), np.uint8)
        _check(load_library().gm_msm_prepared(self.handle, curve_id(curve), int(g2), scalars.ptr, prepared.ptr, n,
                                              _p(jac), _p(aff)))
        return jac.tobytes(), aff.tobytes()

    def points_upload_precomputed(self, curve, points, g2: bool = False, window: int = 0) -> DeviceBuffer:
        """Point set plus its fixed-base window copies (gm_points_upload_precomputed)."""
        a = _buf(points)
        n = a.size // point_bytes(curve, g2)
        p = ctypes.c_void_p()
        _check(load_library().gm_points_upload_precomputed(self.handle, curve_id(curve), int(g2), _p(a), n, window,
                                                           ctypes.byref(p)))
        buf = DeviceBuffer(self, p.value, a.size)
        buf.count = n
        buf.window = window
        return buf

    def msm_precomputed(self, curve, scalars: DeviceBuffer, prepared: DeviceBuffer, n: int, g2: bool = False):
        jac = np.zeros(jac_bytes(curve, g2), np.uint8)
        aff = np.zeros(point_bytes(curve, g2), np.uint8)
        _check(load_library().gm_msm_precomputed(self.handle, curve_id(curve), int(g2), scalars.ptr, prepared.ptr,
                                                 prepared.count, prepared.window, n, _p(jac), _p(aff)))
        return jac.tobytes(), aff.tobytes()

    def kzg_commit(self, curve, srs: DeviceBuffer, coeffs) -> bytes:
        """kzg.Commit(p, pk): G1 digest of the polynomial coefficients (host)."""
        c = _buf(coeffs)
        out = np.zeros(point_bytes(curve, False), np.uint8)
        _check(load_library().gm_kzg_commit(self.handle, curve_id(curve), srs.ptr, srs.count, _p(c),
                                            c.size // FR_BYTES, _p(out)))
        return out.tobytes()

    def msm_on_device(self, scalars, points, n, curve="bn254"):
        """MsmOnDevice(scalars_d, points_d, count, convert=true) -> G1Jac bytes."""
        return self.msm(curve, scalars, points, n, g2=False)[0]

    def msm_g2_on_device(self, scalars, points, n, curve="bn254"):
        """MsmG2OnDevice -> G2Jac bytes."""
        return self.msm(curve, scalars, points, n, g2=True)[0]

    # ---- NTT -----------------------------------------------------------------
    def ntt(self, curve, data: DeviceBuffer, n: int, inverse: bool, dit: bool, coset: bool):
        _check(load_library().gm_ntt(self.handle, curve_id(curve), data.ptr, n, int(inverse), int(dit),
                                     int(coset)))

    def generate_twiddle_factors(self, curve, n: int, inverse: bool = False):
        """Twiddle tables are built and cached per (curve, n) inside the context on
        first use; this warms that cache (GenerateTwiddleFactors)."""
        tmp = self.malloc(FR_BYTES * n)
        try:
            _check(load_library().gm_ntt(self.handle, curve_id(curve), tmp.ptr, n, int(inverse), 0, 0))
        finally:
            tmp.free()

    # ---- iciclegnark call-for-call binding (icicle.go:68-76,489-510) ----------
    def icicle_generate_twiddle_factors(self, curve, n: int, inverse: bool) -> DeviceBuffer:
        """GenerateTwiddleFactors: a freeable handle; the tables live in the context."""
        p = ctypes.c_void_p()
        _check(load_library().gm_icicle_generate_twiddles(self.handle, curve_id(curve), n, int(inverse),
                                                          ctypes.byref(p)))
        return DeviceBuffer(self, p.value, 64)

    def icicle_intt_on_device(self, curve, scalars: DeviceBuffer, n: int, is_coset: bool) -> DeviceBuffer:
        """INttOnDevice: natural evaluations -> NEW buffer of natural coefficients."""
        p = ctypes.c_void_p()
        _check(load_library().gm_icicle_intt_on_device(self.handle, curve_id(curve), scalars.ptr, n, int(is_coset),
                                                       ctypes.byref(p)))
        return DeviceBuffer(self, p.value, FR_BYTES * n)

    def icicle_ntt_on_device(self, curve, out: DeviceBuffer, scalars: DeviceBuffer, n: int, is_coset: bool):
        """NttOnDevice(out, in): natural coefficients -> natural evaluations in out."""
        _check(load_library().gm_icicle_ntt_on_device(self.handle, curve_id(curve), out.ptr, scalars.ptr, n,
                                                      int(is_coset)))

    def icicle_poly_ops(self, curve, a: DeviceBuffer, b: DeviceBuffer, c: DeviceBuffer, den: DeviceBuffer, n: int):
        """PolyOps(a, b, c, den_d, n) with a device den vector."""
        _check(load_library().gm_icicle_poly_ops(self.handle, curve_id(curve), a.ptr, b.ptr, c.ptr, den.ptr, n))

    def poly_ops(self, curve, a: DeviceBuffer, b: DeviceBuffer, c: DeviceBuffer, n: int, den: bytes):
        d = _buf(den)
        _check(load_library().gm_poly_ops(self.handle, curve_id(curve), a.ptr, b.ptr, c.ptr, n, _p(d)))

    def reverse_scalars(self, curve, data: DeviceBuffer, n: int):
        _check(load_library().gm_reverse_scalars(self.handle, curve_id(curve), data.ptr, n))

    def compute_h(self, curve, a: DeviceBuffer, b: DeviceBuffer, c: DeviceBuffer, length: int, n: int):
        _check(load_library().gm_groth16_compute_h(self.handle, curve_id(curve), a.ptr, b.ptr, c.ptr,
                                                   length, n))

    # ---- synthetic inputs ---------------------------------------------------
    def random_scalars(self, curve, n: int, seed: int) -> DeviceBuffer:
        buf = self.malloc(FR_BYTES * n)
        _check(load_library().gm_random_scalars(self.handle, curve_id(curve), seed, n, buf.ptr))
        return buf

    def batch_mul_base(self, curve, g2: bool, base: bytes, scalars: DeviceBuffer, n: int) -> DeviceBuffer:
        out = self.malloc(point_bytes(curve, g2) * n)
        b = _buf(base)
        _check(load_library().gm_batch_mul_base(self.handle, curve_id(curve), int(g2), _p(b), scalars.ptr,
                                                n, out.ptr))
        return out


    # ---- test hooks ---------------------------------------------------------
    def test_field_op(self, curve, kind: int, op: int, a: bytes, b: bytes) -> bytes:
        A, B = self.copy_to_device(a), self.copy_to_device(b)
        O = self.malloc(len(a))
        esz = {0: 32, 1: FP_BYTES[curve_id(curve)], 2: 2 * FP_BYTES[curve_id(curve)]}[kind]
        try:
            _check(load_testhooks().gm_test_field_op(self.handle, curve_id(curve), kind, op, A.ptr, B.ptr, O.ptr,
                                                   len(a) // esz))
            return O.to_host()
        finally:
            for x in (A, B, O):
                x.free()

    def test_point_op(self, curve, g2: bool, op: int, a: bytes, b: bytes) -> bytes:
        A, B = self.copy_to_device(a), self.copy_to_device(b)
        O = self.malloc(len(a))
        try:
            _check(load_testhooks().gm_test_point_op(self.handle, curve_id(curve), int(g2), op, A.ptr, B.ptr,
                                                   O.ptr, len(a) // point_bytes(curve, g2)))
            return O.to_host()
        finally:
            for x in (A, B, O):
                x.free()


# ---------------------------------------------------------------------------
# Multi-GPU MSM sharding: one process per GPU, each rank owns a
# contiguous slice of the point / scalar arrays, computes its partial Pippenger
# sum, and the N partial Jacobians (96 B G1 / 192 B G2 for BN254) are
# all-gathered (RCCL over xGMI with backend "nccl", or gloo on CPU) and reduced
# by N-1 host EC adds.  No other data-path communication.
# ---------------------------------------------------------------------------
def shard_range(n: int, world: int, rank: int) -> tuple[int, int]:
    """[lo, hi) of the contiguous shard of n items owned by `rank` (the first
    n % world ranks hold one extra item; a shard may be empty)."""
    if world <= 0 or not 0 <= rank < world:
        raise ValueError("bad rank/world")
    q, r = divmod(n, world)
    lo = rank * q + min(rank, r)
    return lo, lo + q + (1 if rank < r else 0)


def jac_infinity(curve, g2: bool) -> bytes:
    """gnark's G1Jac/G2Jac point at infinity {X: 1, Y: 1, Z: 0} (Montgomery one)."""
    out = np.zeros(jac_bytes(curve, g2), np.uint8)
    one = _mont_one(curve, g2)
    out[:one.size] = one
    out[one.size:2 * one.size] = one
    return out.tobytes()


_MONT_ONE_CACHE: dict = {}


def _mont_one(curve, g2: bool) -> np.ndarray:
    """Montgomery encoding of 1 in Fp (or Fp2 = (1, 0)), gnark layout."""
    key = (curve_id(curve), g2)
    if key not in _MONT_ONE_CACHE:
        cid = curve_id(curve)
        p = {BN254: 21888242871839275222246405745257275088696311157297823662689037894645226208583,
             BLS12_377: 258664426012969094010652733694893533536393512754914660539884262666720468348340822774968888139573360124440321458177}[cid]
        nb = FP_BYTES[cid]
        r = (1 << (8 * nb)) % p
        v = np.frombuffer(r.to_bytes(nb, "little"), np.uint8)
        if g2:
            v = np.concatenate([v, np.zeros(nb, np.uint8)])
        _MONT_ONE_CACHE[key] = v
    return _MONT_ONE_CACHE[key]


def reduce_partials(curve, g2: bool, partials) -> bytes:
    """Sum of gnark Jacobian partial results (host EC adds)."""
    acc = None
    for p in partials:
        acc = bytes(p) if acc is None else jac_add(curve, g2, acc, p)
    return acc if acc is not None else jac_infinity(curve, g2)


def allgather_partial(local_jac: bytes, group=None, device=None) -> list:
    """All-gathers one Jacobian partial (fixed size) from every rank."""
    import torch
    import torch.distributed as dist
    dev = device if device is not None else ("cuda" if dist.get_backend(group) == "nccl" else "cpu")
    t = torch.frombuffer(bytearray(local_jac), dtype=torch.uint8).to(dev)
    parts = [torch.empty_like(t) for _ in range(dist.get_world_size(group))]
    dist.all_gather(parts, t, group=group)
    return [q.cpu().numpy().tobytes() for q in parts]


def sharded_msm(ctx: "Context", curve, scalars, points, n_local: int, g2: bool = False, group=None,
                device=None) -> bytes:
    """Full MSM over the union of every rank's shard: local Pippenger on this
    rank's GPU, one all-gather of the partial sums, host reduction.  Returns the
    gnark Jacobian bytes (identical on every rank)."""
    if n_local:
        local = ctx.msm(curve, scalars, points, n_local, g2=g2)[0]
    else:
        local = jac_infinity(curve, g2)
    return reduce_partials(curve, g2, allgather_partial(local, group=group, device=device))


# ---------------------------------------------------------------------------
# Groth16 (icicle_bn254 ProvingKey / Prove mirror)
# ---------------------------------------------------------------------------
class _PkHost(ctypes.Structure):
    _fields_ = [(k, ctypes.c_size_t) for k in ["domain_size", "nb_wires", "nb_public", "nbA", "nbB", "nbK"]] + \
               [(k, ctypes.c_void_p) for k in ["g1_alpha", "g1_beta", "g1_delta", "g1_A", "g1_B", "g1_Z", "g1_K",
                                                "g2_beta", "g2_delta", "g2_B", "infA", "infB", "k_wires"]]


def _pk_host_struct(curve, pk: dict, domain_size: int, nb_wires: int, nb_public: int, shard=None,
                    pk_is_shard: bool = False):
    """gm_g16_pk_host for `pk` (a dict of gnark-layout arrays, see ProvingKey).
    shard = (rank, world): point arrays are sliced to the rank's shard unless
    pk_is_shard (they already are; the counts then come from pk['shard_sizes'])."""
    g1b, g2b = point_bytes(curve, False), point_bytes(curve, True)
    keys = ("g1_alpha", "g1_beta", "g1_delta", "g1_A", "g1_B", "g1_Z", "g1_K", "g2_beta", "g2_delta", "g2_B",
            "infA", "infB")
    arrs = {k: _buf(pk[k]) for k in keys}
    h = _PkHost()
    h.domain_size, h.nb_wires, h.nb_public = domain_size, nb_wires, nb_public
    if pk_is_shard:
        h.nbA, h.nbB, h.nbK = pk["shard_sizes"]
    else:
        h.nbA = arrs["g1_A"].size // g1b
        h.nbB = arrs["g1_B"].size // g1b
        h.nbK = arrs["g1_K"].size // g1b
    if "k_wires" in pk and pk["k_wires"] is not None:
        kw = np.ascontiguousarray(np.asarray(pk["k_wires"], dtype=np.uint32))
        h.nbK = kw.size
        h.k_wires = kw.ctypes.data
        arrs["k_wires"] = kw
    if shard is not None and not pk_is_shard:
        rank, world = shard
        for key, count, pb in (("g1_A", h.nbA, g1b), ("g1_B", h.nbB, g1b), ("g1_K", h.nbK, g1b),
                               ("g1_Z", domain_size - 1, g1b), ("g2_B", h.nbB, g2b)):
            lo, hi = shard_range(count, world, rank)
            arrs[key] = arrs[key][pb * lo:pb * hi].copy() if hi > lo else np.zeros(pb, np.uint8)
    for k in ["g1_alpha", "g1_beta", "g1_delta", "g1_A", "g1_B", "g1_Z", "g1_K", "g2_beta", "g2_delta",
              "g2_B", "infA", "infB"]:
        setattr(h, k, arrs[k].ctypes.data)
    return h, arrs


class ProvingKey:
    """Device-resident Groth16 proving key (icicle_bn254.ProvingKey + deviceInfo,
    provingkey.go:10-28; uploaded once like setupDevicePointers, icicle.go:31-130).

    `pk` is a dict of gnark-layout byte arrays: g1_alpha, g1_beta, g1_delta, g1_A,
    g1_B, g1_Z (n-1, bit-reversed), g1_K, g2_beta, g2_delta, g2_B, infA, infB, and
    optionally k_wires (the wire index of each pk.G1.K point when BSB22
    commitments filter K, prove.go:243-245; default nb_public + i).

    shard = (rank, world) keeps only this rank's slice of every point array on
    the device (gm_g16_pk_upload_shard; sharded_prove); with pk_is_shard the
    point arrays in `pk` already are the slices and pk['shard_sizes'] = (nbA, nbB, nbK)
    gives the whole key's counts.
    """

    PRECOMPUTE = 1  # GM_PK_PRECOMPUTE
    PRECOMPUTE_AUTO = 2  # GM_PK_PRECOMPUTE_AUTO: window copies iff they fit the device

    @classmethod
    def _flags(cls, precompute):
        """precompute: False / True / "auto" (GM_PK_PRECOMPUTE_AUTO)."""
        if precompute == "auto":
            return cls.PRECOMPUTE_AUTO
        return cls.PRECOMPUTE if precompute else 0

    @property
    def precomputed(self) -> bool:
        """Whether the device key holds the window copies (the auto choice)."""
        v = ctypes.c_int()
        _check(load_library().gm_g16_pk_precomputed(self.handle, ctypes.byref(v)))
        return bool(v.value)

    def __init__(self, ctx: Context, curve, pk: dict, domain_size: int, nb_wires: int, nb_public: int,
                 precompute: bool = False, shard=None, pk_is_shard: bool = False):
        self.ctx = ctx
        self.curve = curve_id(curve)
        h, arrs = _pk_host_struct(curve, pk, domain_size, nb_wires, nb_public, shard, pk_is_shard)
        self._keep = arrs
        self._h = h
        handle = ctypes.c_void_p()
        flags = self._flags(precompute)
        rank, world = shard if shard is not None else (0, 1)
        _check(load_library().gm_g16_pk_upload_shard(ctx.handle, self.curve, ctypes.byref(h), flags, rank, world,
                                                     ctypes.byref(handle)))
        self.handle = handle
        self.n, self.nb_wires, self.nb_public = domain_size, nb_wires, nb_public
        self.shard = (rank, world)

    @classmethod
    def from_dump(cls, ctx: Context, curve, path: str, offset: int, meta: dict, domain_size: int, nb_wires: int,
                  nb_public: int, precompute: bool = False, shard=None):
        """Streams the point slices of a gnark WriteDump file (marshal.go:389-456)
        from byte `offset` into device buffers (gm_g16_pk_upload_dump_shard).
        `meta` holds the header fields (g1_alpha, g1_beta, g1_delta, g2_beta,
        g2_delta, infA, infB, optional k_wires) and the counts nbA / nbB / nbK.
        Returns (key, end_offset)."""
        self = cls.__new__(cls)
        self.ctx = ctx
        self.curve = curve_id(curve)
        g1b, g2b = point_bytes(curve, False), point_bytes(curve, True)
        stub = dict(meta)
        for k, pb in (("g1_A", g1b), ("g1_B", g1b), ("g1_Z", g1b), ("g1_K", g1b), ("g2_B", g2b)):
            stub[k] = np.zeros(pb, np.uint8)
        counts = stub.pop("counts")
        h, arrs = _pk_host_struct(curve, stub, domain_size, nb_wires, nb_public)
        h.nbA, h.nbB = counts[0], counts[1]
        if not ("k_wires" in meta and meta["k_wires"] is not None):
            h.nbK = counts[2]
        self._keep, self._h = arrs, h
        handle, end = ctypes.c_void_p(), ctypes.c_uint64()
        rank, world = shard if shard is not None else (0, 1)
        fd = os.open(path, os.O_RDONLY)
        try:
            _check(load_library().gm_g16_pk_upload_dump_shard(ctx.handle, self.curve, ctypes.byref(h),
                                                              fd, offset, cls._flags(precompute),
                                                              rank, world, ctypes.byref(end), ctypes.byref(handle)))
        finally:
            os.close(fd)
        self.handle = handle
        self.n, self.nb_wires, self.nb_public = domain_size, nb_wires, nb_public
        self.shard = (rank, world)
        return self, end.value

    def save_cache(self, path: str):
        """Device-layout copy of this key (gm_g16_pk_save_cache)."""
        fd = os.open(path, os.O_WRONLY | os.O_CREAT | os.O_TRUNC, 0o644)
        try:
            _check(load_library().gm_g16_pk_save_cache(self.ctx.handle, self.handle, fd))
        finally:
            os.close(fd)

    @classmethod
    def from_cache(cls, ctx: Context, path: str, like: "ProvingKey" = None):
        """Key read back from save_cache (gm_g16_pk_load_cache); `like` supplies
        the host-side metadata (the host finishing only needs what the cache holds)."""
        self = cls.__new__(cls)
        self.ctx = ctx
        handle = ctypes.c_void_p()
        fd = os.open(path, os.O_RDONLY)
        try:
            _check(load_library().gm_g16_pk_load_cache(ctx.handle, fd, ctypes.byref(handle)))
        finally:
            os.close(fd)
        self.handle = handle
        if like is not None:
            self.curve, self._h, self._keep = like.curve, like._h, like._keep
            self.n, self.nb_wires, self.nb_public, self.shard = like.n, like.nb_wires, like.nb_public, like.shard
        return self

    def stage(self, nb_constraints: int) -> "Stage":
        return Stage(self, nb_constraints)

    def free(self):
        if self.handle:
            load_library().gm_g16_pk_free(self.ctx.handle, self.handle)
            self.handle = None

    def prove(self, wires, a, b, c, r: bytes, s: bytes):
        """Returns (Ar, Bs, Krs) affine bytes (gnark layout)."""
        W, A, B, C, R, S = (_buf(x) for x in (wires, a, b, c, r, s))
        ar = np.zeros(point_bytes(self.curve, False), np.uint8)
        krs = np.zeros(point_bytes(self.curve, False), np.uint8)
        bs = np.zeros(point_bytes(self.curve, True), np.uint8)
        _check(load_library().gm_g16_prove(self.ctx.handle, self.handle, _p(W), _p(A), _p(B), _p(C),
                                           A.size // FR_BYTES, _p(R), _p(S), _p(ar), _p(bs), _p(krs)))
        return ar.tobytes(), bs.tobytes(), krs.tobytes()

    def prove_r1cs(self, r1cs: "R1CS", wires, r: bytes, s: bytes):
        """gm_g16_prove_r1cs: the wires are the only host input; a, b, c come
        from the device-resident constraint system."""
        W, R, S = (_buf(x) for x in (wires, r, s))
        ar = np.zeros(point_bytes(self.curve, False), np.uint8)
        krs = np.zeros(point_bytes(self.curve, False), np.uint8)
        bs = np.zeros(point_bytes(self.curve, True), np.uint8)
        _check(load_library().gm_g16_prove_r1cs(self.ctx.handle, self.handle, r1cs.handle, _p(W), _p(R), _p(S),
                                                _p(ar), _p(bs), _p(krs)))
        return ar.tobytes(), bs.tobytes(), krs.tobytes()

    def prove_device(self, wires: DeviceBuffer, a: DeviceBuffer, b: DeviceBuffer, c: DeviceBuffer,
                     nb_constraints: int, r: bytes, s: bytes):
        R, S = _buf(r), _buf(s)
        ar = np.zeros(point_bytes(self.curve, False), np.uint8)
        krs = np.zeros(point_bytes(self.curve, False), np.uint8)
        bs = np.zeros(point_bytes(self.curve, True), np.uint8)
        _check(load_library().gm_g16_prove_device(self.ctx.handle, self.handle, wires.ptr, a.ptr, b.ptr, c.ptr,
                                                  nb_constraints, _p(R), _p(S), _p(ar), _p(bs), _p(krs)))
        return ar.tobytes(), bs.tobytes(), krs.tobytes()

    def prove_partial_device(self, wires: DeviceBuffer, a: DeviceBuffer, b: DeviceBuffer, c: DeviceBuffer,
                             nb_constraints: int) -> bytes:
        """This shard's raw MSM sums (gm_g16_prove_partial): 4 G1Jac + 1 G2Jac."""
        out = np.zeros(g16_partial_bytes(self.curve), np.uint8)
        _check(load_library().gm_g16_prove_partial(self.ctx.handle, self.handle, wires.ptr, a.ptr, b.ptr, c.ptr,
                                                   nb_constraints, _p(out)))
        return out.tobytes()


class PendingMsm:
    def __init__(self, handle, curve, g2):
        self.handle, self.curve, self.g2 = handle, curve, g2

    def wait(self):
        jac = np.zeros(jac_bytes(self.curve, self.g2), np.uint8)
        aff = np.zeros(point_bytes(self.curve, self.g2), np.uint8)
        h, self.handle = self.handle, None
        _check(load_library().gm_msm_wait(h, _p(jac), _p(aff)))
        return jac.tobytes(), aff.tobytes()


class Stage:
    """Prover inputs handed over while Solve runs (gm_g16_stage_*): put_range /
    put_indexed per solver level (constraint/bn254/solver.go:426-532), then prove."""

    A, B, C, WIRES = 0, 1, 2, 3

    def __init__(self, pk: ProvingKey, nb_constraints: int):
        self.pk = pk
        h = ctypes.c_void_p()
        _check(load_library().gm_g16_stage_begin(pk.ctx.handle, pk.handle, nb_constraints, ctypes.byref(h)))
        self.handle = h

    def put_range(self, which: int, lo: int, data):
        d = _buf(data)
        _check(load_library().gm_g16_stage_put_range(self.handle, which, lo, d.size // FR_BYTES, _p(d)))

    def put_indexed(self, which: int, base, idx):
        b = _buf(base)
        ix = np.ascontiguousarray(np.asarray(idx, dtype=np.uint32))
        _check(load_library().gm_g16_stage_put_indexed(self.handle, which, _p(b), ix.ctypes.data, ix.size))

    def replay_chain(self, wires, nb_inputs: int, nb_constraints: int, abc=None, coalesce=True,
                     flush_at: int = 1 << 16) -> float:
        """Test hook (gm_test_stage_replay_chain): stages the squaring chain's
        level shape -- level j finishes constraint j and solves wire nb_inputs + j
        -- one put per level (coalesce=False) or gathered as the Go level hook
        does.  abc = (a, b, c) host vectors to stage as well.  Returns host ns per
        level."""
        w = _buf(wires)
        bufs = [_buf(x) for x in abc] if abc is not None else []
        ptrs = [_p(x) for x in bufs] if bufs else [None, None, None]
        ns = ctypes.c_double()
        _check(load_testhooks().gm_test_stage_replay_chain(self.handle, _p(w), nb_inputs, ptrs[0], ptrs[1], ptrs[2],
                                                           nb_constraints, 1 if coalesce else 0, 1 if bufs else 0,
                                                           flush_at, ctypes.byref(ns)))
        return ns.value

    def prove(self, r: bytes, s: bytes):
        R, S = _buf(r), _buf(s)
        ar = np.zeros(point_bytes(self.pk.curve, False), np.uint8)
        krs = np.zeros(point_bytes(self.pk.curve, False), np.uint8)
        bs = np.zeros(point_bytes(self.pk.curve, True), np.uint8)
        _check(load_library().gm_g16_stage_prove(self.handle, _p(R), _p(S), _p(ar), _p(bs), _p(krs)))
        return ar.tobytes(), bs.tobytes(), krs.tobytes()

    def prove_r1cs(self, r1cs: "R1CS", r: bytes, s: bytes):
        """gm_g16_stage_prove_r1cs: the wires were staged (during Solve), a, b, c
        come from the device-resident constraint system."""
        R, S = _buf(r), _buf(s)
        ar = np.zeros(point_bytes(self.pk.curve, False), np.uint8)
        krs = np.zeros(point_bytes(self.pk.curve, False), np.uint8)
        bs = np.zeros(point_bytes(self.pk.curve, True), np.uint8)
        _check(load_library().gm_g16_stage_prove_r1cs(self.handle, r1cs.handle, _p(R), _p(S), _p(ar), _p(bs),
                                                      _p(krs)))
        return ar.tobytes(), bs.tobytes(), krs.tobytes()

    def free(self):
        if self.handle:
            load_library().gm_g16_stage_free(self.handle)
            self.handle = None


def write_dump_slices(path: str, curve, pk: dict, prefix: bytes = b"") -> int:
    """Writes `prefix` then pk's five point arrays as gnark-crypto
    utils/unsafe.WriteSlice records in WriteDump order (marshal.go:430-444):
    u64 little-endian count + raw points.  Returns the offset of the first
    slice.  (Test / tooling helper: the real file comes from gnark's WriteDump.)"""
    with open(path, "wb") as f:
        f.write(prefix)
        for key, g2 in (("g1_A", False), ("g1_B", False), ("g1_Z", False), ("g1_K", False), ("g2_B", True)):
            raw = _buf(pk[key]).tobytes()
            f.write(struct.pack("<Q", len(raw) // point_bytes(curve, g2)))
            f.write(raw)
    return len(prefix)


class Multi:
    """Several devices driven from ONE process (gm_multi): one context and host
    thread per entry of device_ids (entries may repeat: several contexts on one
    GPU rehearse the multi-GPU path).  The single-process seam gnark's
    groth16.Prove needs (backend/groth16/groth16.go:192-204)."""

    def __init__(self, device_ids):
        ids = (ctypes.c_int * len(device_ids))(*device_ids)
        h = ctypes.c_void_p()
        _check(load_library().gm_multi_init(ids, len(device_ids), ctypes.byref(h)))
        self.handle = h
        self.device_ids = list(device_ids)

    def close(self):
        if self.handle:
            load_library().gm_multi_destroy(self.handle)
            self.handle = None

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()


R1CS_CONST = 0xFFFFFFFF  # GM_R1CS_CONST: a constant term (constraint.Term.IsConstant)


class R1CS:
    """A constraint system resident on the device (gm_r1cs_upload): per matrix
    L, R, O a CSR of (coefficient id, wire id) terms over a coefficient table
    (gnark's CoeffTable: id 0 = 0, 1 = 1, 2 = 2, 3 = -1, 4 = -2, then the
    circuit's own).  from_terms builds the table from per-term coefficients."""

    def __init__(self, ctx: Context, curve, nb_constraints: int, nb_wires: int, rowptr, cid, vid, coeffs: bytes):
        self.ctx = ctx
        self.curve = curve_id(curve)
        self.nc, self.nb_wires = nb_constraints, nb_wires
        rp = [np.ascontiguousarray(np.asarray(x, np.uint32)) for x in rowptr]
        ci = [np.ascontiguousarray(np.asarray(x if len(x) else [0], np.uint32)) for x in cid]
        vi = [np.ascontiguousarray(np.asarray(x if len(x) else [0], np.uint32)) for x in vid]
        co = _buf(coeffs)
        arr = lambda xs: (ctypes.c_void_p * 3)(*[x.ctypes.data for x in xs])
        handle = ctypes.c_void_p()
        _check(load_library().gm_r1cs_upload(ctx.handle, self.curve, nb_constraints, nb_wires, arr(rp), arr(ci),
                                             arr(vi), _p(co), co.size // FR_BYTES, ctypes.byref(handle)))
        self.handle = handle

    @classmethod
    def from_terms(cls, ctx: Context, curve, nb_constraints: int, nb_wires: int, rowptr, wires, coeffs, modulus: int):
        """rowptr / wires / coeffs per matrix as in tests/r1cs.R1CS (coeffs: 32-byte
        Montgomery values per term)."""
        R = (1 << 256) % modulus
        enc = lambda v: (v * R % modulus).to_bytes(32, "little")
        table = [enc(0), enc(1), enc(2), enc(modulus - 1), enc(modulus - 2)]
        index = {t: k for k, t in enumerate(table)}
        cid = []
        for m in range(3):
            cb = bytes(np.asarray(coeffs[m], np.uint8).tobytes())
            nt = int(rowptr[m][-1])
            ids = []
            for q in range(nt):
                t = cb[32 * q:32 * q + 32]
                if t not in index:
                    index[t] = len(table)
                    table.append(t)
                ids.append(index[t])
            cid.append(ids)
        vid = [list(np.asarray(wires[m], np.uint32)[:int(rowptr[m][-1])]) for m in range(3)]
        return cls(ctx, curve, nb_constraints, nb_wires, rowptr, cid, vid, b"".join(table))

    def eval(self, wires: DeviceBuffer, a: DeviceBuffer, b: DeviceBuffer, c: DeviceBuffer):
        _check(load_library().gm_r1cs_eval(self.ctx.handle, self.handle, wires.ptr, a.ptr, b.ptr, c.ptr))

    def free(self):
        if self.handle:
            load_library().gm_r1cs_free(self.ctx.handle, self.handle)
            self.handle = None


class ProvingKeyMulti:
    """A proving key sharded across the devices of a Multi (gm_g16_pk_upload_multi)."""

    def __init__(self, multi: Multi, curve, pk: dict, domain_size: int, nb_wires: int, nb_public: int,
                 precompute: bool = False):
        self.multi = multi
        self.curve = curve_id(curve)
        h, arrs = _pk_host_struct(curve, pk, domain_size, nb_wires, nb_public)
        self._keep, self._h = arrs, h
        handle = ctypes.c_void_p()
        _check(load_library().gm_g16_pk_upload_multi(multi.handle, self.curve, ctypes.byref(h),
                                                     ProvingKey.PRECOMPUTE if precompute else 0,
                                                     ctypes.byref(handle)))
        self.handle = handle

    def free(self):
        if self.handle:
            load_library().gm_g16_pk_free_multi(self.multi.handle, self.handle)
            self.handle = None

    def prove(self, wires, a, b, c, r: bytes, s: bytes):
        """(Ar, Bs, Krs) affine bytes; wires / a / b / c in host memory."""
        W, A, B, C, R, S = (_buf(x) for x in (wires, a, b, c, r, s))
        ar = np.zeros(point_bytes(self.curve, False), np.uint8)
        krs = np.zeros(point_bytes(self.curve, False), np.uint8)
        bs = np.zeros(point_bytes(self.curve, True), np.uint8)
        _check(load_library().gm_g16_prove_multi(self.multi.handle, self.handle, _p(W), _p(A), _p(B), _p(C),
                                                 A.size // FR_BYTES, _p(R), _p(S), _p(ar), _p(bs), _p(krs)))
        return ar.tobytes(), bs.tobytes(), krs.tobytes()


def device_count() -> int:
    n = ctypes.c_int()
    _check(load_library().gm_device_count(ctypes.byref(n)))
    return n.value


def g16_partial_bytes(curve) -> int:
    n = ctypes.c_size_t()
    _check(load_library().gm_g16_partial_bytes(curve_id(curve), ctypes.byref(n)))
    return n.value


def g16_reduce_partials(curve, partials) -> bytes:
    """Component-wise host sum of rank partials [A, B, K, Z (G1Jac), B2 (G2Jac)]."""
    j1, j2 = jac_bytes(curve, False), jac_bytes(curve, True)
    out = []
    for k in range(5):
        g2 = k == 4
        lo = 4 * j1 if g2 else k * j1
        sz = j2 if g2 else j1
        out.append(reduce_partials(curve, g2, [bytes(p)[lo:lo + sz] for p in partials]))
    return b"".join(out)


def g16_finish(curve, pk_host: "_PkHost", sums: bytes, r: bytes, s: bytes):
    """(Ar, Bs, Krs) affine bytes from summed partials (gm_g16_finish, host only)."""
    S, R, SS = _buf(sums), _buf(r), _buf(s)
    ar = np.zeros(point_bytes(curve, False), np.uint8)
    krs = np.zeros(point_bytes(curve, False), np.uint8)
    bs = np.zeros(point_bytes(curve, True), np.uint8)
    _check(load_library().gm_g16_finish(curve_id(curve), ctypes.byref(pk_host), _p(S), _p(R), _p(SS), _p(ar),
                                        _p(bs), _p(krs)))
    return ar.tobytes(), bs.tobytes(), krs.tobytes()


def sharded_prove(pk: ProvingKey, wires: DeviceBuffer, a: DeviceBuffer, b: DeviceBuffer, c: DeviceBuffer,
                  nb_constraints: int, r: bytes, s: bytes, group=None, device=None):
    """Multi-GPU Groth16 prove (BASELINE config 4): every rank computes its
    shard's five MSM sums, the fixed-size partials are all-gathered (RCCL over
    xGMI for backend "nccl", gloo on CPU) and every rank sums them and applies
    the blinding on the host.  Returns (Ar, Bs, Krs) on every rank."""
    local = pk.prove_partial_device(wires, a, b, c, nb_constraints)
    parts = allgather_partial(local, group=group, device=device)
    return g16_finish(pk.curve, pk._h, g16_reduce_partials(pk.curve, parts), r, s)
