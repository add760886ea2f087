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
