#!/usr/bin/env python3
"""Where the staged prove's fixed overhead comes from: the
same key and inputs proved through gm_g16_prove_device and gm_g16_stage_prove /
gm_g16_stage_prove_r1cs, each timed right after the previous GPU work and after
an idle pause of the length bench.py's staged scopes sleep ("the staged copies
finish during Solve").  An idle GPU lowers its clocks; if the gap follows the
pause rather than the API, it is the clock ramp, not the staged path.

  python3 tools/staged_overhead.py [logn=20] [reps=5] [idle_ms=50]
"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "gnark-icicle_amd"))
import numpy as np  # noqa: E402
import bench  # noqa: E402
import gnark_mi355x as gm  # noqa: E402


def main():
    logn = int(sys.argv[1]) if len(sys.argv) > 1 else 20
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 5
    idle = (int(sys.argv[3]) if len(sys.argv) > 3 else 50) / 1e3
    ctx = gm.Context(0)
    n = 1 << logn
    nbw = n + 2
    pk = bench.synthetic_pk(ctx, gm, n, nbw, 2)
    dpk = gm.ProvingKey(ctx, "bn254", pk, n, nbw, 2, precompute=False)
    W = ctx.random_scalars("bn254", nbw, 8)
    srcs = [ctx.random_scalars("bn254", n, 9 + i) for i in range(3)]
    r = ctx.random_scalars("bn254", 2, 12).to_host()
    host = [np.frombuffer(x.to_host(), np.uint8) for x in [W] + srcs]
    A, B, C = (ctx.malloc(32 * n) for _ in range(3))
    ch = bench.chain_r1cs(ctx, gm, n, nbw)

    def device(pause):
        for dst, src in zip((A, B, C), srcs):
            dst.copy_from(src)
        ctx.synchronize()
        if pause:
            time.sleep(idle)
        t0 = time.perf_counter()
        p = dpk.prove_device(W, A, B, C, n, r[:32], r[32:])
        return time.perf_counter() - t0, p

    def staged(pause, r1cs):
        st = dpk.stage(n)
        st.put_range(st.WIRES, 0, host[0])
        if not r1cs:
            for which, v in ((st.A, host[1]), (st.B, host[2]), (st.C, host[3])):
                st.put_range(which, 0, v)
        ctx.synchronize()
        if pause:
            time.sleep(idle)
        t0 = time.perf_counter()
        p = st.prove_r1cs(ch, r[:32], r[32:]) if r1cs else st.prove(r[:32], r[32:])
        dt = time.perf_counter() - t0
        st.free()
        return dt, p

    def r1cs_dev(pause):
        ctx.synchronize()
        if pause:
            time.sleep(idle)
        t0 = time.perf_counter()
        p = dpk.prove_r1cs(ch, host[0], r[:32], r[32:])
        return time.perf_counter() - t0, p

    cases = [("device", lambda p: device(p)), ("staged", lambda p: staged(p, False)),
             ("r1cs_host_wires", lambda p: r1cs_dev(p)), ("staged_r1cs", lambda p: staged(p, True))]
    for name, fn in cases:  # warm-up (arenas, stage buffers, pinned rings)
        fn(False)
    res = {}
    for rep in range(reps):
        for pause in (False, True):
            for name, fn in cases:
                dt, _ = fn(pause)
                res.setdefault((name, pause), []).append(dt * 1e3)
    print("2^%d, %d reps, idle pause %.0f ms (median / min ms):" % (logn, reps, idle * 1e3))
    for (name, pause), v in res.items():
        v.sort()
        print("  %-16s %-10s %8.3f %8.3f" % (name, "after-idle" if pause else "busy", v[len(v) // 2], v[0]))
    ch.free()
    dpk.free()
    ctx.close()


if __name__ == "__main__":
    main()
