#!/usr/bin/env python3
"""Generates the committed golden fixtures in tests/golden/ from the pure-Python
restatement oracle/pyref.py (fixed seeds; independent of the C++ oracle and of
the HIP library, both of which are checked against these files).

The reference tree holds no MSM / NTT / H known-answer vectors,
so these vectors are restatement outputs: they pin the C++ oracle and the GPU
path to the big-integer restatement, not to gnark-crypto itself.

Run:  python tests/golden/make_golden.py
"""
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", "..", "oracle"))
sys.path.insert(0, os.path.join(HERE, ".."))
import pyref  # noqa: E402
import r1cs as R  # noqa: E402


def hx(b: bytes) -> str:
    return b.hex()


def msm_case(cname, g2, n, seed):
    c = pyref.CURVES[cname]
    G = pyref.Group(c, g2)
    pts = pyref.random_points(c, n, seed, g2)
    sc = pyref.random_scalars(c, n, seed + 1)
    pts[1] = None
    sc[2], sc[3], sc[4] = 0, 1, c.r - 1
    pts[6], sc[6] = pts[5], sc[5]
    pts[8], sc[8] = G.neg(pts[7]), sc[7]
    return {
        "curve": cname, "g2": g2, "n": n, "seed": seed,
        "scalars": hx(b"".join(pyref.encode_fr(c, s) for s in sc)),
        "points": hx(b"".join(pyref.encode_point(c, p, g2) for p in pts)),
        "expected_affine": hx(pyref.encode_point(c, G.msm(sc, pts), g2)),
    }


def ntt_case(cname, n, seed):
    c = pyref.CURVES[cname]
    vals = pyref.random_scalars(c, n, seed)
    out = {"curve": cname, "n": n, "seed": seed,
           "input": hx(b"".join(pyref.encode_fr(c, v) for v in vals)), "outputs": {}}
    for inverse in (0, 1):
        for dit in (0, 1):
            for coset in (0, 1):
                fn = pyref.fft_inverse if inverse else pyref.fft
                res = fn(c, vals, "DIT" if dit else "DIF", bool(coset))
                out["outputs"]["%d%d%d" % (inverse, dit, coset)] = hx(b"".join(pyref.encode_fr(c, v) for v in res))
    return out


def h_case(cname, circ, W):
    c = pyref.CURVES[cname]
    a, b, cc = circ.solve_abc(W)
    h = pyref.compute_h(c, a, b, cc, circ.domain_size)
    enc = lambda v: hx(b"".join(pyref.encode_fr(c, x) for x in v))
    return {"curve": cname, "n": circ.domain_size, "a": enc(a), "b": enc(b), "c": enc(cc), "h_bitrev": enc(h)}


def g16_case(cname, circ, W, toxic, r_, s_):
    c = pyref.CURVES[cname]
    pk = pyref.g16_setup(c, circ.cons, circ.nb_wires, circ.nb_public, toxic)
    a, b, cc = circ.solve_abc(W)
    ar, bs, krs = pyref.g16_prove(c, pk, W, a, b, cc, r_, s_)
    ep = lambda P, g2=False: hx(pyref.encode_point(c, P, g2))
    epl = lambda L, g2=False: hx(b"".join(pyref.encode_point(c, P, g2) for P in L))
    enc = lambda v: hx(b"".join(pyref.encode_fr(c, x) for x in v))
    return {
        "curve": cname, "n": pk["n"], "nb_wires": circ.nb_wires, "nb_public": circ.nb_public,
        "toxic": enc(toxic), "r": enc([r_]), "s": enc([s_]), "wires": enc(W),
        "a": enc(a), "b": enc(b), "c": enc(cc),
        "pk": {"g1_alpha": ep(pk["g1_alpha"]), "g1_beta": ep(pk["g1_beta"]), "g1_delta": ep(pk["g1_delta"]),
               "g1_A": epl(pk["g1_A"]), "g1_B": epl(pk["g1_B"]), "g1_Z": epl(pk["g1_Z"]), "g1_K": epl(pk["g1_K"]),
               "g2_beta": ep(pk["g2_beta"], True), "g2_delta": ep(pk["g2_delta"], True),
               "g2_B": epl(pk["g2_B"], True),
               "infA": hx(bytes(int(x) for x in pk["infA"])), "infB": hx(bytes(int(x) for x in pk["infB"]))},
        "expected": {"Ar": ep(ar), "Bs": ep(bs, True), "Krs": ep(krs)},
    }


def main():
    out = {}
    for cname, g2, n in [("bn254", False, 64), ("bn254", True, 32), ("bls12377", False, 32), ("bls12377", True, 16)]:
        out["msm_%s_%s" % (cname, "g2" if g2 else "g1")] = msm_case(cname, g2, n, 4242 + n + g2)
    for cname in ("bn254", "bls12377"):
        out["ntt_%s" % cname] = ntt_case(cname, 16, 99)
        r1, W = R.cubic_circuit(cname)
        out["h_cubic_%s" % cname] = h_case(cname, r1, W)
        r1, W = R.squaring_chain(15, cname)
        out["h_squaring15_%s" % cname] = h_case(cname, r1, W)
    toxic = [0x1D5A2B3C4D5E6F70, 0x2E6B3C4D5E6F7081, 0x3F7C4D5E6F708192, 0x0A8D5E6F708192A3, 0x1B9E6F708192A3B4]
    r1, W = R.cubic_circuit("bn254")
    out["groth16_cubic_bn254"] = g16_case("bn254", r1, W, toxic, 0x1234567, 0x7654321)
    r1, W = R.cubic_circuit("bls12377")
    out["groth16_cubic_bls12377"] = g16_case("bls12377", r1, W, toxic, 0x1234567, 0x7654321)
    for k, v in out.items():
        with open(os.path.join(HERE, k + ".json"), "w") as f:
            json.dump(v, f, indent=1)
    print("wrote", len(out), "fixtures")


if __name__ == "__main__":
    main()
