#!/usr/bin/env python3
"""Which earlier step of the bench slows a later 2^24 host-input Groth16 prove
(r04q: 167 ms alone, 199 ms after the 2^20 Groth16 section)?  Keeps one 2^24
plain key and its host inputs, and after each candidate step measures the prove
with host inputs (median of 2) and a pageable 512 MiB H2D copy."""
import os
import sys
import time

os.environ.setdefault("GPU_MAX_HW_QUEUES", "8")
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
buf = ctx.malloc(512 << 20)
blob = np.frombuffer(os.urandom(512 << 20), np.uint8)


def probe(tag):
    ctx.synchronize()
    t = []
    for _ in range(3):
        t0 = time.perf_counter()
        buf.write(blob)
        ctx.synchronize()
        t.append(time.perf_counter() - t0)
    p = []
    dpk.prove(host[0], host[1], host[2], host[3], r[:32], r[32:])
    for _ in range(2):
        ctx.synchronize()
        t0 = time.perf_counter()
        dpk.prove(host[0], host[1], host[2], host[3], r[:32], r[32:])
        p.append(time.perf_counter() - t0)
    print("%-28s h2d %6.1f GB/s   prove(host inputs) %7.1f ms" % (tag, (512 << 20) / min(t) / 1e9, sorted(p)[0] * 1e3),
          flush=True)


probe("fresh")
# the 2^20 section, piece by piece
n20 = 1 << 20
pk20 = bench.synthetic_pk(ctx, gm, n20, n20 + 2, 2)
d20 = gm.ProvingKey(ctx, "bn254", pk20, n20, n20 + 2, 2, precompute=False)
W20 = ctx.random_scalars("bn254", n20 + 2, 8)
s20 = [ctx.random_scalars("bn254", n20, 9 + i) for i in range(3)]
h20 = [np.frombuffer(x.to_host(), np.uint8) for x in [W20] + s20]
for _ in range(4):
    d20.prove(h20[0], h20[1], h20[2], h20[3], r[:32], r[32:])
probe("after 2^20 host proves")
proof = d20.prove(h20[0], h20[1], h20[2], h20[3], r[:32], r[32:])
for _ in range(3):
    st = d20.stage(n20)
    for lo in range(0, n20, n20 // 64):
        for which, v in ((st.A, h20[1]), (st.B, h20[2]), (st.C, h20[3])):
            st.put_range(which, lo, v[32 * lo:32 * (lo + n20 // 64)])
    st.put_range(st.WIRES, 0, h20[0])
    ctx.synchronize()
    st.prove(r[:32], r[32:])
    st.free()
probe("after staged proves")
import tempfile  # noqa: E402
meta = {k: pk20[k] for k in ("g1_alpha", "g1_beta", "g1_delta", "g2_beta", "g2_delta", "infA", "infB")}
meta["counts"] = (n20 + 2, n20 + 2, n20)
with tempfile.TemporaryDirectory() as d:
    path = os.path.join(d, "pk.dump")
    off = gm.write_dump_slices(path, "bn254", pk20, b"\0" * 4096)
    k2, _ = gm.ProvingKey.from_dump(ctx, "bn254", path, off, meta, n20, n20 + 2, 2)
    k2.prove(h20[0], h20[1], h20[2], h20[3], r[:32], r[32:])
    probe("after dump upload")
    cpath = os.path.join(d, "pk.cache")
    k2.save_cache(cpath)
    k3 = gm.ProvingKey.from_cache(ctx, cpath, like=k2)
    k3.prove(h20[0], h20[1], h20[2], h20[3], r[:32], r[32:])
    k2.free()
    k3.free()
probe("after cache save/load")
