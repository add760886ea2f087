#!/usr/bin/env python3
"""Groth16 device-input proves only (synthetic key, bench.synthetic_pk) -- the
program behind same-box A/Bs of the prove (tools/ab_run.sh with alternative
library builds via GNARK_MI355X_LIB) and its rocprofv3 timelines / PMC passes.

  python3 tools/g16_only.py [--logn 24] [--precompute] [--reps 3]
"""
import argparse
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "gnark-icicle_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--logn", type=int, default=24)
    ap.add_argument("--precompute", action="store_true")
    ap.add_argument("--reps", type=int, default=3)
    a = ap.parse_args()
    import bench
    import gnark_mi355x as gm
    n = 1 << a.logn
    nbw = n + 2
    with gm.Context(0) as ctx:
        pk = bench.synthetic_pk(ctx, gm, n, nbw, 2)
        dpk = gm.ProvingKey(ctx, "bn254", pk, n, nbw, 2, precompute=a.precompute)
        W = ctx.random_scalars("bn254", nbw, 8)
        srcs = [ctx.random_scalars("bn254", n, 9 + i) for i in range(3)]
        r = ctx.random_scalars("bn254", 2, 12).to_host()
        A, B, C = (ctx.malloc(32 * n) for _ in range(3))
        ts, proof = [], None
        for i in range(a.reps + 1):
            for dst, src in zip((A, B, C), srcs):
                dst.copy_from(src)
            ctx.synchronize()
            t0 = time.perf_counter()
            p = dpk.prove_device(W, A, B, C, n, r[:32], r[32:])
            if i:
                ts.append((time.perf_counter() - t0) * 1e3)
            assert proof is None or p == proof
            proof = p
        ts.sort()
        print("g16 2^%d %s device inputs: median %.2f ms  min %.2f ms  (%s) proof %s" % (
            a.logn, "precomputed" if a.precompute else "plain", ts[len(ts) // 2], ts[0],
            " ".join("%.2f" % t for t in ts), proof[0][:8].hex()), flush=True)
        dpk.free()


if __name__ == "__main__":
    main()
