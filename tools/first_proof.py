#!/usr/bin/env python3
"""Time to first proof in a fresh process -- what a gnark process that proves
once pays (the reference uploads the key lazily inside the
first Prove, backend/groth16/bn254/icicle/icicle.go:145-150 -> :31-130):
library load + context, the key streamed from a WriteDump file
(gm_g16_pk_upload_dump, marshal.go:389-456) or read back from a device-layout
cache (gm_g16_pk_load_cache), then the first and a second host-input prove.

  python3 tools/first_proof.py INPUTS.npz DUMP_OR_CACHE OFFSET PRECOMPUTE(0|1|auto|cache)

INPUTS.npz (written by bench.py): the key's header fields (g1_alpha, g1_beta,
g1_delta, g2_beta, g2_delta, infA, infB), counts, domain_size, nb_wires,
nb_public and the proof inputs W, a, b, c, r.  Prints one JSON line.
"""
import json
import os
import sys
import time

T_START = time.perf_counter()
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "gnark-icicle_amd"))
import numpy as np  # noqa: E402
import gnark_mi355x as gm  # noqa: E402


def main():
    inputs, path, offset, mode = sys.argv[1], sys.argv[2], int(sys.argv[3]), sys.argv[4]
    z = np.load(inputs)  # plain arrays only (allow_pickle stays False)
    n, nbw, nbp = (int(z[k]) for k in ("domain_size", "nb_wires", "nb_public"))
    meta = {k: z[k] for k in ("g1_alpha", "g1_beta", "g1_delta", "g2_beta", "g2_delta", "infA", "infB")}
    meta["counts"] = tuple(int(x) for x in z["counts"])
    W, a, b, c, r = (z[k].tobytes() for k in ("W", "a", "b", "c", "r"))
    t0 = time.perf_counter()
    gm.load_library()
    ctx = gm.Context(0)
    t_ctx = time.perf_counter()
    if mode == "cache":
        like = gm.ProvingKey.__new__(gm.ProvingKey)
        stub = dict(meta)
        g1b, g2b = gm.point_bytes("bn254", False), gm.point_bytes("bn254", True)
        for k, pb in (("g1_A", g1b), ("g1_B", g1b), ("g1_Z", g1b), ("g1_K", g1b), ("g2_B", g2b)):
            stub[k] = np.zeros(pb, np.uint8)
        stub.pop("counts")
        like._h, like._keep = gm._pk_host_struct("bn254", stub, n, nbw, nbp)
        like._h.nbA, like._h.nbB, like._h.nbK = meta["counts"]
        like.curve, like.n, like.nb_wires, like.nb_public, like.shard = gm.curve_id("bn254"), n, nbw, nbp, (0, 1)
        dpk = gm.ProvingKey.from_cache(ctx, path, like=like)
    else:
        pre = {"0": False, "1": True, "auto": "auto"}[mode]
        dpk, _ = gm.ProvingKey.from_dump(ctx, "bn254", path, offset, meta, n, nbw, nbp, precompute=pre)
    t_up = time.perf_counter()
    proof = dpk.prove(W, a, b, c, r[:32], r[32:])
    t_first = time.perf_counter()
    proof2 = dpk.prove(W, a, b, c, r[:32], r[32:])
    t_second = time.perf_counter()
    print(json.dumps({"mode": mode, "precomputed": bool(dpk.precomputed),
                      "imports_s": round(t0 - T_START, 3), "lib_and_context_s": round(t_ctx - t0, 3),
                      "pk_upload_s": round(t_up - t_ctx, 3), "first_prove_ms": round((t_first - t_up) * 1e3, 1),
                      "second_prove_ms": round((t_second - t_first) * 1e3, 1),
                      "to_first_proof_s": round(t_first - T_START, 3), "proofs_equal": proof == proof2,
                      "proof_hex": "".join(x.hex() for x in proof)}))
    dpk.free()
    ctx.close()


if __name__ == "__main__":
    main()
