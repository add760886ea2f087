"""The drop-in boundary (include/gnark_mi355x.h) without a GPU: the shared
library builds for gfx950, loads, and exports every entry point the header
declares.  No compute call is made."""
import ctypes
import os
import re
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "gnark_mi355x.h")
TEST_HEADER = os.path.join(ROOT, "include", "gnark_mi355x_testhooks.h")
LIB = os.path.join(ROOT, "gnark-icicle_amd", "libgnark_mi355x.so")
TLIB = os.path.join(ROOT, "gnark-icicle_amd", "libgnark_mi355x_testhooks.so")


def _declared(header=HEADER):
    src = open(header).read()
    return sorted(set(re.findall(r"\b(gm_[a-z0-9_]+)\s*\(", src)))


@pytest.fixture(scope="module")
def lib():
    if not os.path.exists(LIB):
        subprocess.check_call(["make", "-s", "-j8", "-C", os.path.join(ROOT, "gnark-icicle_amd")])
    return ctypes.CDLL(LIB)


def test_header_declares_entry_points():
    names = _declared()
    for must in ("gm_init", "gm_msm", "gm_ntt", "gm_poly_ops", "gm_reverse_scalars", "gm_groth16_compute_h",
                 "gm_g16_prove", "gm_copy_to_device", "gm_copy_points_to_device", "gm_free"):
        assert must in names


def test_library_exports_every_declared_symbol(lib):
    missing = [n for n in _declared() if not hasattr(lib, n)]
    assert not missing, missing


def test_python_binding_symbol_list_matches_header():
    import gnark_mi355x as gm
    assert sorted(gm.SYMBOLS) == _declared()
    assert sorted(gm.TEST_SYMBOLS) == _declared(TEST_HEADER)


def test_test_hooks_live_outside_the_product_library(lib):
    """The element-wise test hooks are a separate test-only library; the product
    library exports none of them."""
    tests_only = _declared(TEST_HEADER)
    assert tests_only and not set(tests_only) & set(_declared())
    assert not [n for n in tests_only if hasattr(lib, n)]
    assert os.path.exists(TLIB)
    t = ctypes.CDLL(TLIB)
    assert all(hasattr(t, n) for n in tests_only)
    nm = subprocess.run(["nm", "-D", "--defined-only", LIB], capture_output=True, text=True).stdout
    assert "k_field_op" not in nm and "k_point_op" not in nm


def test_library_leaves_process_environment_alone():
    """Loading the library changes no process-wide HIP setting (the
    earlier load-time GPU_MAX_HW_QUEUES default depended on load order and
    reached every other HIP user in the process)."""
    import sys
    code = ("import ctypes, sys; ctypes.CDLL(sys.argv[1]); libc = ctypes.CDLL(None); "
            "libc.getenv.restype = ctypes.c_char_p; print(libc.getenv(b'GPU_MAX_HW_QUEUES'))")
    env = {k: v for k, v in os.environ.items() if k != "GPU_MAX_HW_QUEUES"}
    out = subprocess.run([sys.executable, "-c", code, LIB], env=env, capture_output=True, text=True, check=True)
    assert out.stdout.strip() == "None"
    env["GPU_MAX_HW_QUEUES"] = "4"
    out = subprocess.run([sys.executable, "-c", code, LIB], env=env, capture_output=True, text=True, check=True)
    assert out.stdout.strip() == "b'4'"


def test_host_helpers_without_gpu(lib):
    """Host-only entry points work without a device: generator table and the
    Jacobian helpers used for finishing adds (gm_jac_add, gm_jac_to_affine)."""
    import gnark_mi355x as gm
    import pyref
    for cname in ("bn254", "bls12377"):
        c = pyref.CURVES[cname]
        for g2 in (False, True):
            G = pyref.Group(c, g2)
            gen = gm.generator(cname, g2)
            assert pyref.decode_point(c, gen, g2) == G.generator()
            n = gm.FP_BYTES[gm.curve_id(cname)] * (2 if g2 else 1)
            one = pyref.encode_point(c, ((1, 0), (0, 0)) if g2 else (1, 0), g2)[:n]
            jac = gen + one  # (X, Y, Z=1)
            two = gm.jac_add(cname, g2, jac, jac)
            assert pyref.decode_point(c, gm.jac_to_affine(cname, g2, two), g2) == G.mul(G.generator(), 2)


def test_precompute_layout_host_only(lib):
    """gm_precompute_layout is pure host logic: window choice and copy count."""
    c, w = ctypes.c_int(), ctypes.c_int()
    lib.gm_precompute_layout.argtypes = [ctypes.c_int, ctypes.c_size_t, ctypes.c_int,
                                         ctypes.POINTER(ctypes.c_int), ctypes.POINTER(ctypes.c_int)]
    assert lib.gm_precompute_layout(0, 1 << 20, 0, ctypes.byref(c), ctypes.byref(w)) == 0
    assert (c.value, w.value) == (20, 13)
    assert lib.gm_precompute_layout(0, 1 << 24, 0, ctypes.byref(c), ctypes.byref(w)) == 0
    assert (c.value, w.value) == (22, 12)
    assert lib.gm_precompute_layout(1, 1000, 9, ctypes.byref(c), ctypes.byref(w)) == 0
    assert (c.value, w.value) == (9, 29)   # ceil((253 + 1) / 9)
    assert lib.gm_precompute_layout(0, 1000, 40, ctypes.byref(c), ctypes.byref(w)) != 0
    assert lib.gm_precompute_layout(7, 1000, 0, ctypes.byref(c), ctypes.byref(w)) != 0
