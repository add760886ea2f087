#!/usr/bin/env python3
"""Runs only NTTs (no tests, no oracle) -- the program profiled by rocprofv3
--pmc passes and per-kernel A/Bs of the NTT.

  python tools/ntt_only.py [--curve bn254] [--logn 24] [--reps 5] [--coset]
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
    ap.add_argument("--logn", type=int, default=24)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--coset", action="store_true")
    a = ap.parse_args()
    import gnark_mi355x as gm
    n = 1 << a.logn
    with gm.Context(0) as ctx:
        X = ctx.random_scalars(a.curve, n, 7)
        ctx.ntt(a.curve, X, n, False, False, a.coset)  # domain tables (untimed)
        ctx.ntt(a.curve, X, n, True, True, a.coset)
        ctx.synchronize()
        ctx.profile(True)
        ctx.profile_reset()
        t0 = time.perf_counter()
        for _ in range(a.reps):
            ctx.ntt(a.curve, X, n, False, False, a.coset)
            ctx.ntt(a.curve, X, n, True, True, a.coset)
        ctx.synchronize()
        dt = (time.perf_counter() - t0) / (2 * a.reps)
        st = ctx.profile_stats()
        ks = " ".join("%s=%.4f" % (k, v[0] / max(v[1], 1)) for k, v in sorted(st.items()))
        print("%s ntt 2^%d%s: %.4f ms/transform  %.3f Gelem/s | %s" % (
            a.curve, a.logn, " coset" if a.coset else "", dt * 1e3, n / dt / 1e9, ks), flush=True)
        X.free()


if __name__ == "__main__":
    main()
