"""Multi-rank MSM sharding on CPU (gloo, world_size 2 and 3): the N>1 path of
bench.py / SURVEY.md §8e.  Each rank computes the partial MSM of its contiguous
shard (here with the CPU oracle, standing in for its GPU), the partial Jacobians
are all-gathered, and the host reduction must equal the single-process MSM of
the whole array.  Exercises the real gather/reduce code of gnark_mi355x
(shard_range, allgather_partial, reduce_partials) and the C-ABI host adds."""
import os
import socket

import numpy as np
import pytest

import pyref

torch = pytest.importorskip("torch")
import torch.distributed as dist  # noqa: E402
import torch.multiprocessing as mp  # noqa: E402


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _jac_from_affine(gm, cname, g2, aff: bytes) -> bytes:
    if aff == bytes(len(aff)):
        return gm.jac_infinity(cname, g2)
    return aff + bytes(gm._mont_one(cname, g2))  # {x, y, 1}


def _worker(rank, world, port, cname, g2, n, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import gnark_mi355x as gm
        import oracle_lib
        c = pyref.CURVES[cname]
        vals = pyref.random_scalars(c, n, 77)
        sc = b"".join(pyref.encode_fr(c, v) for v in vals)
        pts = oracle_lib.batch_mul_base(cname, g2, oracle_lib.generator(cname, g2),
                                        b"".join(pyref.encode_fr(c, v) for v in pyref.random_scalars(c, n, 78)))
        pb = gm.point_bytes(cname, g2)
        lo, hi = gm.shard_range(n, world, rank)
        if hi > lo:
            aff = oracle_lib.msm(cname, g2, sc[32 * lo:32 * hi], pts[pb * lo:pb * hi], nthreads=1)
            local = _jac_from_affine(gm, cname, g2, aff)
        else:
            local = gm.jac_infinity(cname, g2)
        parts = gm.allgather_partial(local, device="cpu")
        assert len(parts) == world
        total = gm.reduce_partials(cname, g2, parts)
        got = gm.jac_to_affine(cname, g2, total)
        exp = oracle_lib.msm(cname, g2, sc, pts, nthreads=1)
        q.put((rank, got == exp))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("cname,g2,n,world", [("bn254", False, 1000, 2), ("bn254", True, 257, 2),
                                               ("bls12377", False, 300, 3), ("bn254", False, 1, 2)])
def test_sharded_msm_gloo(cname, g2, n, world):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, cname, g2, n, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in procs]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert sorted(res) == [(r, True) for r in range(world)]


def test_shard_range_partitions():
    import gnark_mi355x as gm
    for n in (0, 1, 7, 8, 1 << 20):
        for world in (1, 2, 3, 8):
            spans = [gm.shard_range(n, world, r) for r in range(world)]
            assert spans[0][0] == 0 and spans[-1][1] == n
            assert all(a[1] == b[0] for a, b in zip(spans, spans[1:]))
            sizes = [h - l for l, h in spans]
            assert max(sizes) - min(sizes) <= 1


def test_jac_infinity_is_identity():
    import gnark_mi355x as gm
    import oracle_lib
    for cname in ("bn254", "bls12377"):
        for g2 in (False, True):
            g = oracle_lib.generator(cname, g2)
            gj = g + bytes(gm._mont_one(cname, g2))
            inf = gm.jac_infinity(cname, g2)
            assert gm.jac_to_affine(cname, g2, gm.jac_add(cname, g2, gj, inf)) == g
            assert gm.jac_to_affine(cname, g2, gm.reduce_partials(cname, g2, [inf, gj, inf])) == g
            assert gm.jac_to_affine(cname, g2, inf) == bytes(len(g))


TOXIC = [0x1D5A2B3C4D5E6F708192A3B4C5D6E7F8091A2B3C4D5E6F708192A3B4C5D6E7,
         0x2E6B3C4D5E6F708192A3B4C5D6E7F8091A2B3C4D5E6F708192A3B4C5D6E7F8,
         0x3F7C4D5E6F708192A3B4C5D6E7F8091A2B3C4D5E6F708192A3B4C5D6E7F809,
         0x0A8D5E6F708192A3B4C5D6E7F8091A2B3C4D5E6F708192A3B4C5D6E7F8091A,
         0x1B9E6F708192A3B4C5D6E7F8091A2B3C4D5E6F708192A3B4C5D6E7F8091A2B]


def _g16_worker(rank, world, port, cname, k, q):
    """One rank of the sharded Groth16 prove (BASELINE config 4): its five
    partial MSM sums over its pk slices (the CPU oracle standing in for its GPU),
    all-gathered, reduced and finished by the product's host code
    (gnark_mi355x.g16_reduce_partials / gm_g16_finish)."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import gnark_mi355x as gm
        import oracle_lib
        import r1cs as R
        c = pyref.CURVES[cname]
        r1, W = R.squaring_chain(k, cname, x=3)
        tox = R.encode_vec(cname, [t % c.r for t in TOXIC])
        pk = oracle_lib.g16_setup(cname, r1, tox)
        a, b, cc = r1.solve_abc(W)
        enc = lambda v: R.encode_vec(cname, v)
        wires = np.frombuffer(enc(W), np.uint8).reshape(-1, 32)
        rb, sb = enc([0x1111]), enc([0x2222])
        n = r1.domain_size
        h = np.frombuffer(oracle_lib.compute_h(cname, enc(a), enc(b), enc(cc), n, nthreads=1),
                          np.uint8).reshape(-1, 32)
        idxA = np.nonzero(pk["infA"] == 0)[0]
        idxB = np.nonzero(pk["infB"] == 0)[0]
        idxK = np.arange(r1.nb_public, r1.nb_wires)
        g1b, g2b = gm.point_bytes(cname, False), gm.point_bytes(cname, True)

        def part(g2, scal, pts, pb):
            lo, hi = gm.shard_range(len(scal), world, rank)
            if hi == lo:
                return gm.jac_infinity(cname, g2)
            aff = oracle_lib.msm(cname, g2, scal[lo:hi].tobytes(), pts[pb * lo:pb * hi], nthreads=1)
            if aff == bytes(len(aff)):
                return gm.jac_infinity(cname, g2)
            return aff + bytes(gm._mont_one(cname, g2))

        local = b"".join([part(False, wires[idxA], pk["g1_A"].tobytes(), g1b),
                          part(False, wires[idxB], pk["g1_B"].tobytes(), g1b),
                          part(False, wires[idxK], pk["g1_K"].tobytes(), g1b),
                          part(False, h[: n - 1], pk["g1_Z"].tobytes(), g1b),
                          part(True, wires[idxB], pk["g2_B"].tobytes(), g2b)])
        assert len(local) == gm.g16_partial_bytes(cname)
        parts = gm.allgather_partial(local, device="cpu")
        hs, _keep = gm._pk_host_struct(cname, pk, n, r1.nb_wires, r1.nb_public)
        got = gm.g16_finish(cname, hs, gm.g16_reduce_partials(cname, parts), rb, sb)
        exp = oracle_lib.g16_prove(cname, pk, r1.nb_public, enc(W), enc(a), enc(b), enc(cc), rb, sb, nthreads=1)
        q.put((rank, got == exp))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("cname,k,world", [("bn254", 255, 2), ("bls12377", 100, 3)])
def test_sharded_groth16_gloo(cname, k, world):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_g16_worker, args=(r, world, port, cname, k, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=180) for _ in procs]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert sorted(res) == [(r, True) for r in range(world)]
