"""Proving-key I/O and staged inputs, each checked
by proving with the key / inputs it produced and comparing byte for byte with
the oracle's groth16_bn254.Prove restatement (prove.go:62-325) on the same pk,
witness and (r, s).

* gm_g16_pk_upload_dump: the five point slices of a WriteDump file
  (marshal.go:389-456: utils/unsafe.WriteSlice records -- u64 LE count + raw
  points) streamed from a file; the dump here is written by
  gnark_mi355x.write_dump_slices behind an opaque header of the test's own
  (gnark's real header is parsed by the Go side; only its length matters here).
* gm_g16_pk_save_cache / gm_g16_pk_load_cache: device-layout round trip (plain
  and GM_PK_PRECOMPUTE keys).
* gm_g16_stage_*: a, b, c handed over in random "solver levels" (index lists)
  and the wires in ranges, interleaved, then one prove."""
import os

import numpy as np
import pytest

import pyref
import r1cs as R
from test_groth16_gpu import TOXIC

pytestmark = pytest.mark.gpu


def _setup(oracle, cname, k):
    c = pyref.CURVES[cname]
    r1, W = R.squaring_chain(k, cname, x=3)
    tox = R.encode_vec(cname, [t % c.r for t in TOXIC])
    pk = oracle.g16_setup(cname, r1, tox)
    a, b, cc = r1.solve_abc(W)
    enc = lambda v: R.encode_vec(cname, v)
    rb, sb = enc([0x1111ABCDEF]), enc([0x2222FEDCBA])
    exp = oracle.g16_prove(cname, pk, r1.nb_public, enc(W), enc(a), enc(b), enc(cc), rb, sb)
    return r1, pk, (enc(W), enc(a), enc(b), enc(cc)), rb, sb, exp


def _meta(pk):
    import gnark_mi355x as gm
    meta = {k: pk[k] for k in ("g1_alpha", "g1_beta", "g1_delta", "g2_beta", "g2_delta", "infA", "infB")}
    meta["k_wires"] = pk.get("k_wires")
    g1b = len(pk["g1_alpha"])
    meta["counts"] = (len(pk["g1_A"]) // g1b, len(pk["g1_B"]) // g1b, len(pk["g1_K"]) // g1b)
    return meta


@pytest.mark.parametrize("cname,k,precompute,shard", [("bn254", 1023, False, None), ("bn254", 4000, True, None),
                                                      ("bls12377", 511, False, None), ("bn254", 1023, False, (1, 3))])
def test_pk_upload_dump(gm_ctx, oracle, tmp_path, cname, k, precompute, shard):
    import gnark_mi355x as gm
    r1, pk, (W, A, B, C), rb, sb, exp = _setup(oracle, cname, k)
    path = str(tmp_path / "pk.dump")
    header = os.urandom(1234)  # stands in for the marker / Domain / raw header fields
    off = gm.write_dump_slices(path, cname, pk, header)
    dpk, end = gm.ProvingKey.from_dump(gm_ctx, cname, path, off, _meta(pk), r1.domain_size, r1.nb_wires,
                                       r1.nb_public, precompute=precompute, shard=shard)
    try:
        assert end == os.path.getsize(path)
        if shard is None:
            assert dpk.prove(W, A, B, C, rb, sb) == exp
        else:
            # this rank's partial equals the partial of the same shard uploaded from memory
            ref = gm.ProvingKey(gm_ctx, cname, pk, r1.domain_size, r1.nb_wires, r1.nb_public, shard=shard)
            try:
                bufs = []
                for v in (W, A, B, C):
                    x = np.frombuffer(v, np.uint8).copy()
                    n = r1.domain_size * 32 if v is not W else len(v)
                    y = np.zeros(n, np.uint8)
                    y[:len(x)] = x
                    bufs.append(y)
                outs = []
                for key in (dpk, ref):
                    d = [gm_ctx.copy_to_device(y.tobytes()) for y in bufs]
                    outs.append(key.prove_partial_device(d[0], d[1], d[2], d[3], len(A) // 32))
                    for x in d:
                        x.free()
                # Jacobian sums: equal points (the bucket order inside a sum is free)
                j1 = gm.point_bytes(cname, False) // 2 * 3  # one G1Jac
                aff = lambda o: [gm.jac_to_affine(cname, q == 4, o[q * j1:(q + 1) * j1] if q < 4 else o[4 * j1:])
                                 for q in range(5)]
                assert aff(outs[0]) == aff(outs[1])
            finally:
                ref.free()
    finally:
        dpk.free()


def test_pk_dump_rejects_wrong_counts(gm_ctx, oracle, tmp_path):
    import gnark_mi355x as gm
    r1, pk, _, _, _, _ = _setup(oracle, "bn254", 15)
    path = str(tmp_path / "pk.dump")
    off = gm.write_dump_slices(path, "bn254", pk, b"hdr")
    meta = _meta(pk)
    meta["counts"] = (meta["counts"][0] + 1,) + meta["counts"][1:]
    with pytest.raises(gm.GmError, match="slice 0"):
        gm.ProvingKey.from_dump(gm_ctx, "bn254", path, off, meta, r1.domain_size, r1.nb_wires, r1.nb_public)
    with pytest.raises(gm.GmError, match="holds"):  # misplaced offset: a garbage count
        gm.ProvingKey.from_dump(gm_ctx, "bn254", path, off + 40, _meta(pk), r1.domain_size, r1.nb_wires,
                                r1.nb_public)
    os.truncate(path, os.path.getsize(path) - 100)  # G2.B cut short
    with pytest.raises(gm.GmError, match="end of file"):
        gm.ProvingKey.from_dump(gm_ctx, "bn254", path, off, _meta(pk), r1.domain_size, r1.nb_wires, r1.nb_public)


@pytest.mark.parametrize("cname,precompute", [("bn254", False), ("bn254", True), ("bls12377", True)])
def test_pk_cache_round_trip(gm_ctx, oracle, tmp_path, cname, precompute):
    import gnark_mi355x as gm
    r1, pk, (W, A, B, C), rb, sb, exp = _setup(oracle, cname, 1500)
    dpk = gm.ProvingKey(gm_ctx, cname, pk, r1.domain_size, r1.nb_wires, r1.nb_public, precompute=precompute)
    path = str(tmp_path / "pk.cache")
    try:
        dpk.save_cache(path)
        back = gm.ProvingKey.from_cache(gm_ctx, path, like=dpk)
        try:
            assert back.prove(W, A, B, C, rb, sb) == exp
        finally:
            back.free()
    finally:
        dpk.free()
    with open(path, "r+b") as f:
        f.write(b"NOTACACH")
    with pytest.raises(gm.GmError, match="magic"):
        gm.ProvingKey.from_cache(gm_ctx, path)


@pytest.mark.parametrize("cname,k", [("bn254", 4000), ("bls12377", 511)])
def test_staged_inputs_by_level(gm_ctx, oracle, cname, k):
    import gnark_mi355x as gm
    r1, pk, (W, A, B, C), rb, sb, exp = _setup(oracle, cname, k)
    nc = len(A) // 32
    dpk = gm.ProvingKey(gm_ctx, cname, pk, r1.domain_size, r1.nb_wires, r1.nb_public)
    st = dpk.stage(nc)
    try:
        rng = np.random.default_rng(k)
        perm = rng.permutation(nc)
        cuts = np.sort(rng.choice(np.arange(1, nc), size=min(40, nc - 1), replace=False))
        levels = np.split(perm, cuts)  # disjoint index sets covering every constraint
        nw = len(W) // 32
        wcuts = [0] + sorted(rng.choice(np.arange(1, nw), size=min(7, nw - 1), replace=False).tolist()) + [nw]
        for j, lv in enumerate(levels):
            for which, vec in ((st.A, A), (st.B, B), (st.C, C)):
                st.put_indexed(which, vec, lv)
            if j < len(wcuts) - 1:
                lo, hi = wcuts[j], wcuts[j + 1]
                st.put_range(st.WIRES, lo, W[32 * lo:32 * hi])
        for j in range(len(levels), len(wcuts) - 1):
            lo, hi = wcuts[j], wcuts[j + 1]
            st.put_range(st.WIRES, lo, W[32 * lo:32 * hi])
        assert st.prove(rb, sb) == exp
        with pytest.raises(gm.GmError, match="outside"):
            st.put_indexed(st.A, A, [nc])
    finally:
        st.free()
        dpk.free()


@pytest.mark.parametrize("coalesce,flush_at", [(False, 1), (True, 977), (True, 1 << 16)])
def test_staged_squaring_chain_level_shape(gm_ctx, oracle, coalesce, flush_at):
    """The reference benchmark circuit's level shape (groth16_test.go:120-156: a
    chain of squarings, one constraint and one solved wire per solver level,
    solver.go:471-484) staged through gm_g16_stage_put_indexed by the C test
    driver: one put per level and vector, or gathered as the Go level hook does
    (integration/go/icicle_bn254/staged.go, a put every flush_at ids).  The
    small puts share ring slots (records gathered in the open slot).  a, b, c
    and the wires staged -> gm_g16_stage_prove; the wires only with the system
    resident -> gm_g16_stage_prove_r1cs; both equal the oracle's proof."""
    import gnark_mi355x as gm
    k = 3000
    r1, pk, (W, A, B, C), rb, sb, exp = _setup(oracle, "bn254", k)
    nc = len(A) // 32
    assert nc == k + 1 and len(W) // 32 == 3 + k
    dpk = gm.ProvingKey(gm_ctx, "bn254", pk, r1.domain_size, r1.nb_wires, r1.nb_public)
    h = gm.R1CS.from_terms(gm_ctx, "bn254", r1.nc, r1.nb_wires, r1.rowptr, r1.wires, r1.coeffs, r1.c.r)
    try:
        st = dpk.stage(nc)
        try:
            ns = st.replay_chain(W, 3, nc, abc=(A, B, C), coalesce=coalesce, flush_at=flush_at)
            assert ns > 0
            assert st.prove(rb, sb) == exp
        finally:
            st.free()
        st = dpk.stage(nc)
        try:
            st.replay_chain(W, 3, nc, coalesce=coalesce, flush_at=flush_at)
            assert st.prove_r1cs(h, rb, sb) == exp
        finally:
            st.free()
    finally:
        h.free()
        dpk.free()


@pytest.mark.parametrize("reuse", ["1", "0"])
def test_staged_buffers_reused_across_proofs(gm_ctx, oracle, monkeypatch, reuse):
    """gm_g16_stage_free parks the stage's buffers with the key and the next
    gm_g16_stage_begin reuses them (no per-proof allocation): consecutive staged
    proofs on one key -- whole-vector puts, then per-level puts in another order,
    then two stages open at once (one reuses the spare, one is fresh) -- all equal
    the oracle.  GM_G16_STAGE_REUSE=0 gives the same proofs without reuse."""
    import gnark_mi355x as gm
    monkeypatch.setenv("GM_G16_STAGE_REUSE", reuse)
    r1, pk, (W, A, B, C), rb, sb, exp = _setup(oracle, "bn254", 700)
    nc = len(A) // 32
    dpk = gm.ProvingKey(gm_ctx, "bn254", pk, r1.domain_size, r1.nb_wires, r1.nb_public)

    def fill(st, order):
        for lv in np.array_split(order, 9):
            for which, vec in ((st.A, A), (st.B, B), (st.C, C)):
                st.put_indexed(which, vec, lv)
        st.put_range(st.WIRES, 0, W)

    try:
        for order in (np.arange(nc), np.arange(nc)[::-1].copy(), np.random.default_rng(3).permutation(nc)):
            st = dpk.stage(nc)
            try:
                fill(st, order)
                assert st.prove(rb, sb) == exp
            finally:
                st.free()
        s1, s2 = dpk.stage(nc), dpk.stage(nc)
        try:
            fill(s2, np.arange(nc))
            fill(s1, np.arange(nc)[::-1].copy())
            assert s1.prove(rb, sb) == exp and s2.prove(rb, sb) == exp
        finally:
            s1.free()
            s2.free()
    finally:
        dpk.free()


def test_pk_cache_rejects_corrupt_headers_and_indices(gm_ctx, oracle, tmp_path):
    """gm_g16_pk_load_cache checks the header invariants, the device-layout
    fingerprint and every compaction index against the wire slice (k_gather_fr
    reads wires[idx] unchecked), instead of reading a stale / corrupt cache."""
    import struct
    import gnark_mi355x as gm
    r1, pk, (W, A, B, C), rb, sb, exp = _setup(oracle, "bn254", 300)
    dpk = gm.ProvingKey(gm_ctx, "bn254", pk, r1.domain_size, r1.nb_wires, r1.nb_public)
    path = str(tmp_path / "pk.cache")
    try:
        dpk.save_cache(path)
        _corrupt_cache_cases(gm_ctx, gm, dpk, path, r1, (W, A, B, C), rb, sb, exp)
    finally:
        dpk.free()


def _corrupt_cache_cases(gm_ctx, gm, dpk, path, r1, inputs, rb, sb, exp):
    import struct
    W, A, B, C = inputs
    good = open(path, "rb").read()
    HDR = 176  # CacheHeader (pk_io.hip)
    off_n, off_layout, off_wires = 24, 16, 32

    def load_with(blob, match):
        with open(path, "wb") as f:
            f.write(blob)
        with pytest.raises(gm.GmError, match=match):
            gm.ProvingKey.from_cache(gm_ctx, path)

    b = bytearray(good)
    b[off_n:off_n + 8] = struct.pack("<Q", r1.domain_size + 1)
    load_with(bytes(b), "domain size")
    b = bytearray(good)
    b[off_layout:off_layout + 4] = struct.pack("<I", 0xDEAD)
    load_with(bytes(b), "layout")
    b = bytearray(good)
    b[off_wires:off_wires + 8] = struct.pack("<Q", 0)
    load_with(bytes(b), "wire counts")
    # walk to the first compaction map (array 5) and point one entry past the wires
    pos = HDR + 3 * 64 + 2 * 128
    for _ in range(5):
        (sz,) = struct.unpack_from("<Q", good, pos)
        pos += 8 + sz
    (sz,) = struct.unpack_from("<Q", good, pos)
    assert sz > 0
    b = bytearray(good)
    b[pos + 8:pos + 12] = struct.pack("<I", r1.nb_wires)
    load_with(bytes(b), "compaction index")
    with open(path, "wb") as f:
        f.write(good)
    back = gm.ProvingKey.from_cache(gm_ctx, path, like=dpk)
    try:
        assert back.prove(W, A, B, C, rb, sb) == exp
    finally:
        back.free()
