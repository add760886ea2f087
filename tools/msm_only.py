#!/usr/bin/env python3
"""Runs only MSMs (no tests, no oracle) -- the program profiled by rocprofv3
--pmc passes and per-kernel A/Bs.

  python tools/msm_only.py [--curve bn254] [--g2] [--logn 20] [--reps 5] [--window 0]
                           [--scalars uniform|zero|one|wire] [--precompute]
"""
import argparse
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "gnark-icicle_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--curve", default="bn254")
    ap.add_argument("--g2", action="store_true")
    ap.add_argument("--logn", type=int, default=20)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--window", type=int, default=0)
    ap.add_argument("--scalars", default="uniform")
    ap.add_argument("--precompute", action="store_true")
    ap.add_argument("--glv", type=int, default=-1, help="gm_set_msm_glv mode (-1 = the size rule)")
    a = ap.parse_args()
    import numpy as np
    import gnark_mi355x as gm
    n = 1 << a.logn
    with gm.Context(0) as ctx:
        if a.scalars == "uniform":
            S = ctx.random_scalars(a.curve, n, 0x5EED0002)
        else:
            p = {"bn254": 21888242871839275222246405745257275088548364400416034343698204186575808495617,
                 "bls12377": 8444461749428370424248824938781546531375899335154063827935233455917409239041}[a.curve]
            enc = lambda v: (v * (1 << 256) % p).to_bytes(32, "little")
            if a.scalars == "zero":
                sb = bytes(32 * n)
            elif a.scalars == "one":
                sb = enc(1) * n
            else:  # wire-like: {0, 1, 2, r-1}
                t = np.frombuffer(b"".join(enc(v) for v in (0, 1, 2, p - 1)), np.uint8).reshape(4, 32)
                sb = t[np.random.default_rng(1).integers(0, 4, n)].tobytes()
            S = ctx.copy_to_device(sb)
        K = ctx.random_scalars(a.curve, n, 0x5EED1002)
        P = ctx.batch_mul_base(a.curve, a.g2, gm.generator(a.curve, a.g2), K, n)
        K.free()
        ctx.set_msm_window(a.window)
        ctx.set_msm_glv(a.glv)
        if a.precompute:
            pre = ctx.points_upload_precomputed(a.curve, P.to_host(), a.g2, 0)
            run = lambda: ctx.msm_precomputed(a.curve, S, pre, n, g2=a.g2)
        else:
            run = lambda: ctx.msm(a.curve, S, P, n, g2=a.g2)
        run()
        ctx.profile(True)
        ctx.profile_reset()
        ctx.synchronize()
        t0 = time.perf_counter()
        for _ in range(a.reps):
            run()
        dt = (time.perf_counter() - t0) / a.reps
        st = ctx.profile_stats()
        ks = " ".join("%s=%.4f" % (k, v[0] / max(v[1], 1)) for k, v in sorted(st.items()))
        print("%s %s 2^%d %s window=%d glv=%d: %.4f ms/MSM  %.1f Mpoints/s | %s" % (
            a.curve, "g2" if a.g2 else "g1", a.logn, a.scalars, a.window, a.glv, dt * 1e3, n / dt / 1e6, ks), flush=True)


if __name__ == "__main__":
    main()
