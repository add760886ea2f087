#!/usr/bin/env python3
"""2^24 plain-key Groth16 proves with host inputs (the icicle.go:204-412 scope), for a
kernel + memory-copy trace of where the host inputs' cost goes:
  rocprofv3 --kernel-trace --memory-copy-trace ... -- python3 tools/g16_host_trace.py [stage|async|device|devonly]"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "gnark-icicle_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402,F401
import bench  # noqa: E402
import gnark_mi355x as gm  # noqa: E402

ctx = gm.Context(0)
n = 1 << 24
nbw = n + 2
pk = bench.synthetic_pk(ctx, gm, n, nbw, 2)
dpk = gm.ProvingKey(ctx, "bn254", pk, n, nbw, 2, precompute=False)
W = ctx.random_scalars("bn254", nbw, 8)
srcs = [ctx.random_scalars("bn254", n, 9 + i) for i in range(3)]
r = ctx.random_scalars("bn254", 2, 12).to_host()
host = [np.frombuffer(x.to_host(), np.uint8) for x in [W] + srcs]
mode = sys.argv[1] if len(sys.argv) > 1 else ""
if mode == "stage":  # a small staged upload first: pinned copies on the copy stream from this thread
    st = dpk.stage(1 << 10)
    st.put_range(st.A, 0, host[1][:32 << 10])
    ctx.synchronize()
    st.free()
elif mode == "async":  # two pipelined MSMs first: the slot streams come into use
    S = ctx.random_scalars("bn254", 1 << 16, 5)
    P = ctx.batch_mul_base("bn254", False, gm.generator("bn254"), S, 1 << 16)
    a = ctx.msm_async("bn254", S, P, 1 << 16)
    b = ctx.msm_async("bn254", S, P, 1 << 16)
    a.wait()
    b.wait()
elif mode == "device":  # device-input proves first (what bench.py times before the host scope)
    A, B, C = (ctx.malloc(32 * n) for _ in range(3))
    for dst, src in zip((A, B, C), srcs):
        dst.copy_from(src)
    for _ in range(2):
        dpk.prove_device(W, A, B, C, n, r[:32], r[32:])
print("mode", mode or "fresh", flush=True)
if mode in ("devonly", "devonly_ntt"):  # device-input proves only (devonly_ntt: NTT tables built first)
    if mode == "devonly_ntt":
        X = ctx.random_scalars("bn254", n, 3)
        t0 = time.perf_counter()
        ctx.ntt("bn254", X, n, False, False, True)
        ctx.ntt("bn254", X, n, True, True, True)
        ctx.synchronize()
        print("ntt tables + 2 transforms %.1f ms" % ((time.perf_counter() - t0) * 1e3), flush=True)
        X.free()
    A, B, C = (ctx.malloc(32 * n) for _ in range(3))
    for dst, src in zip((A, B, C), srcs):
        dst.copy_from(src)
    Wd = W
    for i in range(3):
        ctx.synchronize()
        t0 = time.perf_counter()
        dpk.prove_device(Wd, A, B, C, n, r[:32], r[32:])
        print("prove(device inputs) %.1f ms" % ((time.perf_counter() - t0) * 1e3), flush=True)
    sys.exit(0)
for i in range(3):
    ctx.synchronize()
    t0 = time.perf_counter()
    dpk.prove(host[0], host[1], host[2], host[3], r[:32], r[32:])
    print("prove(host inputs) %.1f ms" % ((time.perf_counter() - t0) * 1e3), flush=True)
