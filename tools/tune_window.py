#!/usr/bin/env python3
"""Sweep the MSM window size c (gm_set_msm_window) per (curve, group, log n) and
print ms per MSM -- the measurements behind csrc/msm_impl.hpp choose_window.

  python tools/tune_window.py [--cases bn254:g1:20,bn254:g2:20,...] [--reps 3]
"""
import argparse
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "gnark-icicle_amd"))
import gnark_mi355x as gm  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--cases", default="bn254:g1:20,bn254:g2:20,bls12377:g1:22,bls12377:g2:22,bn254:g1:24")
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--span", type=int, default=2)
    args = ap.parse_args()
    ctx = gm.Context(0)
    for case in args.cases.split(","):
        curve, grp, logn = case.split(":")
        g2, logn = grp == "g2", int(logn)
        n = 1 << logn
        S = ctx.random_scalars(curve, n, 1)
        K = ctx.random_scalars(curve, n, 2)
        P = ctx.batch_mul_base(curve, g2, gm.generator(curve, g2), K, n)
        K.free()
        ref = None
        best = None
        base_c = min(20, max(8, logn - 4))
        for c in range(base_c - args.span, base_c + args.span + 1):
            ctx.set_msm_window(c)
            r = ctx.msm(curve, S, P, n, g2=g2)[1]
            ref = ref or r
            assert r == ref, "window %d changed the result" % c
            ctx.synchronize()
            t0 = time.perf_counter()
            for _ in range(args.reps):
                ctx.msm(curve, S, P, n, g2=g2)
            ms = (time.perf_counter() - t0) / args.reps * 1e3
            best = min(best or (ms, c), (ms, c))
            print("%-9s %s 2^%d c=%2d  %8.3f ms" % (curve, grp, logn, c, ms), flush=True)
        print("best %s %s 2^%d: c=%d (%.3f ms)" % (curve, grp, logn, best[1], best[0]), flush=True)
        ctx.set_msm_window(0)
        S.free()
        P.free()
    ctx.close()


if __name__ == "__main__":
    main()
