#!/usr/bin/env python3
"""Benchmark: BN254 G1 MSM throughput (BASELINE.json configs[1]: 2^20 random
points/scalars per GPU) through the C-ABI of libgnark_mi355x.so, plus the
secondary metrics the same BASELINE metric names (NTT Gelem/s at 2^24, Groth16
prove time) on rank 0.

  python bench.py [--gpus N] [--steps K] [--warmup W] [--logn 20]
  torchrun --nproc-per-node N bench.py --gpus N ...   (one rank per GPU)

Multi-GPU = the MSM sharded by splitting the point/scalar array across ranks
(weak scaling: every rank holds a fixed 2^logn shard); each step every rank runs
its shard's Pippenger MSM, the per-rank partial sums (gnark G1Jac, 96 B) are
all-gathered over RCCL and reduced by host EC adds.

Inputs are resident in HBM before the timed region.  The cpu_baseline leg times
the oracle's C++ Pippenger restatement (oracle/, "port", not gnark-crypto: no Go
toolchain on the box) on the same workload on the host.
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "gnark-icicle_amd"))
# MSMs in flight in the step loop (gm_msm_async allows up to 3 per context)
PIPE_DEPTH = int(os.environ.get("GM_BENCH_PIPE_DEPTH", "3"))

HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md chip table (8.0 TB/s spec)
MSM_BYTES_PER_POINT = 96  # 64 B affine point + 32 B scalar
# radix-2^29 BN254 Fp (9 limbs): mul = 2*81 mads, sqr = 45 + 81; the mixed add is
# 8M + 2S with Y3 = R (Q - X3) - Y1 PPP as one reduction of two products (243):
# 6*162 + 2*126 + 243 = 1467 v_mad_u64_u32, the count in the kernel's ISA
# (tools/isa_blocks.py on the hipcc -S listing)
MADS_PER_MIXED_ADD = 6 * 162 + 2 * 126 + 243
# measured v_mad_u64_u32 issue peak: 5.12 cycles per wave64 instruction per SIMD with
# 8 independent chains at 8 waves/SIMD (tools/microbench/isa_rate.hip,
# profiles/r01_isa_rate.txt): 1024 SIMDs x 64 lanes x 2.4 GHz / 5.12 = 30.7 T/s
MAD_PEAK_T = 1024 * 64 * 2.4e9 / 5.12 / 1e12
NTT_BYTES_PER_ELEM = 64   # one 32 B read + one 32 B write per transform
# algorithmic HBM bytes of one config-4 Groth16 prove per domain
# element: 4 x 96 (G1 MSMs) + 160 (G2 MSM) + 7 x 64 (NTT / INTT) + 128 (PolyOps)
G16_BYTES_PER_ELEM = 4 * 96 + 160 + 7 * 64 + 128
# committed rocprofv3 --pmc summaries the roofline's traffic / valu fields are
# read from (collected by tools/gpu_pmc.sh / tools/pmc_traffic.py on the bench's
# own MSM workload; NOT measured inside this run)
PMC_TRAFFIC_FILE = "profiles/r06am_pmc_traffic.json"
PMC_VALU_FILE = "profiles/r06am_pmc_valu.json"
ACCUM_KERNEL = "k_msm_accum_seg_ch"  # the default BN254 G1 accumulation (msm_impl.hpp)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=30)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--logn", type=int, default=20, help="MSM points per GPU = 2^logn")
    ap.add_argument("--ntt-logn", type=int, default=24)
    ap.add_argument("--g16-logn", type=str, default="20,24", help="Groth16 prove domains, comma list ('' = skip)")
    ap.add_argument("--msm-extra", type=int, default=1, help="secondary G2 / BLS12-377 MSM lines (0 = skip)")
    ap.add_argument("--g16-plain", type=str, default="20,24",
                    help="Groth16 domains also proved with a plain (non-precomputed) pk")
    ap.add_argument("--g16-no-precomputed", action="store_true",
                    help="prove only with the plain pk (profiling the default Go path)")
    ap.add_argument("--g16-sharded-logn", type=int, default=24,
                    help="N>1: sharded Groth16 prove domain (BASELINE config 4; 0 = skip)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-secondary", action="store_true")
    return ap.parse_args()


def load_pmc_traffic(name):
    """Fabric bytes per launch of kernel `name` from a committed rocprofv3 --pmc
    summary (tools/pmc_traffic.py), or None: (gather-calibrated bytes, streaming-
    corrected bytes).  FETCH_SIZE tallies 64-byte random gathers 1:1 and
    16-byte-per-lane streaming reads at half their bytes (the calibration in
    profiles/r05f_gather_fetch_calibration.txt), so the accumulation's traffic --
    64-byte point gathers plus 16-byte key / value groups -- lies between
    1024 * FETCH + WRITE and 2 * 1024 * FETCH + WRITE."""
    p = os.path.join(ROOT, PMC_TRAFFIC_FILE)
    try:
        with open(p) as f:
            meta = json.load(f)["_meta"]
        fk = next(v for k, v in meta["fetch_kib"].items() if k == name)
        wk = meta["write_kib"].get(name, 0.0)
        return int(1024 * (fk + wk)), int(1024 * (2 * fk + wk))
    except (OSError, ValueError, KeyError, StopIteration):
        return None


def load_pmc_valu(name):
    """VALU utilisation of a kernel from the committed PMC summary (or None)."""
    p = os.path.join(ROOT, PMC_VALU_FILE)
    try:
        with open(p) as f:
            return json.load(f).get(name)
    except (OSError, ValueError):
        return None


def main():
    args = parse()
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    # torch first (its import does not initialise HIP, and its HIP runtime must be
    # the process's first), then the library.  The bench sets no HIP environment
    # itself, exactly as a gnark process calling the Go hook.
    import torch
    import gnark_mi355x as gm
    hwq_preset = os.environ.get("GPU_MAX_HW_QUEUES")
    gm.load_library()
    dist = None
    if world > 1:
        import torch.distributed as dist
        # one process per GPU; GM_BENCH_BACKEND=gloo (and a device index modulo the
        # visible GPUs) only to rehearse the N>1 code path on a one-GPU box
        local_rank = local_rank % max(torch.cuda.device_count(), 1)
        torch.cuda.set_device(local_rank)
        # the bench's stdout is its one JSON line: whatever the backend prints while the
        # group forms (gloo's "connected to N peer ranks") goes to stderr
        sys.stdout.flush()
        saved_stdout = os.dup(1)
        os.dup2(2, 1)
        try:
            dist.init_process_group(os.environ.get("GM_BENCH_BACKEND", "nccl"))
            dist.barrier()
        finally:
            sys.stdout.flush()
            os.dup2(saved_stdout, 1)
            os.close(saved_stdout)

    ctx = gm.Context(local_rank)
    if os.environ.get("GM_BENCH_MSM_WINDOW"):  # window-size sweeps (0 = the cost model)
        ctx.set_msm_window(int(os.environ["GM_BENCH_MSM_WINDOW"]))
    n = 1 << args.logn
    # ---- resident synthetic inputs: this rank's shard of the MSM ----------------
    seed = 0x5EED0002 + rank
    S = ctx.random_scalars("bn254", n, seed)
    K = ctx.random_scalars("bn254", n, 0x5EED1002 + rank)
    P = ctx.batch_mul_base("bn254", False, gm.generator("bn254"), K, n)
    K.free()
    add_edge_set(ctx, gm, S, P, n)
    ctx.synchronize()

    def barrier():
        if dist is not None:
            dist.barrier()
        torch.cuda.synchronize()

    def step():
        if dist is not None:
            return gm.sharded_msm(ctx, "bn254", S, P, n)
        return ctx.msm("bn254", S, P, n)[0]

    def finish(pend):
        """Host tail of one step: this rank's partial, plus (N > 1) the all-gather
        of every rank's 96-B partial and the host adds -- the full sharded MSM."""
        local = pend.wait()[0]
        if dist is None:
            return local
        return gm.reduce_partials("bn254", False, gm.allgather_partial(local))

    def run(k):
        """k MSMs, pipelined PIPE_DEPTH deep (gm_msm_async, one stream per MSM):
        steps i+1 .. i+PIPE_DEPTH-1 are queued before step i's host tail
        (readback checks + Horner, and at N > 1 the RCCL all-gather of the
        partials and the host adds) runs, so the tail overlaps the GPU and one
        MSM's sort / reduction overlaps another's accumulation; every result is
        complete when run returns."""
        pend, r = [], None
        for _ in range(k):
            pend.append(ctx.msm_async("bn254", S, P, n))
            if len(pend) == PIPE_DEPTH:
                r = finish(pend.pop(0))
        while pend:
            r = finish(pend.pop(0))
        return r

    run(args.warmup)
    # unpipelined latency of one MSM (synchronous gm_msm), for reference; its
    # kernel timings give the accumulation's launch time with nothing beside it
    ctx.profile_reset()
    ctx.profile(True)
    t0 = time.perf_counter()
    for _ in range(3):
        step()
    lat_ms = (time.perf_counter() - t0) / 3 * 1e3
    ctx.profile(False)
    # the accumulation's own execution: first wave start .. last wave end, stamped by
    # its waves (msm_accum_g1_exec, csrc/runtime.hpp ProfScope::wave_stamp); the
    # launch's event brackets (msm_accum_g1) also hold the time it waited for wave
    # slots held by the other MSMs' kernels
    iso_stats = ctx.profile_stats()
    iso_ms, iso_cnt = iso_stats.get("msm_accum_g1_exec", (0.0, 0))
    if not iso_cnt:
        iso_ms, iso_cnt = iso_stats.get("msm_accum_g1", (0.0, 0))
    iso_avg_ms = iso_ms / max(iso_cnt, 1)
    ctx.profile_reset()
    ctx.profile(True)
    barrier()
    t0 = time.perf_counter()
    res = run(args.steps)
    barrier()
    dt = time.perf_counter() - t0
    ctx.profile(False)
    stats = ctx.profile_stats()
    if dist is not None:
        tt = torch.tensor([dt], dtype=torch.float64, device="cuda" if dist.get_backend() == "nccl" else "cpu")
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        dt = float(tt.item())
    ms_per_step = dt * 1e3 / args.steps
    total_points = n * world
    value = total_points / (dt / args.steps) / 1e6

    # ---- roofline of the dominant kernel (bucket accumulation) ------------------
    br_ms, br_cnt = stats.get("msm_accum_g1", (0.0, 0))
    bracket_avg_ms = br_ms / max(br_cnt, 1)
    acc_ms, acc_cnt = stats.get("msm_accum_g1_exec", (0.0, 0))
    stamped = acc_cnt > 0
    if not stamped:
        acc_ms, acc_cnt = br_ms, br_cnt
    acc_avg_ms = acc_ms / max(acc_cnt, 1)
    # A launch time above the step time cannot be the kernel's own run time (the
    # launches would overlap each other): such a figure is not a kernel time and
    # is not priced; the isolated launch (the same kernel with the chip to itself)
    # is used instead and the line says so.
    pipelined_ok = 0 < acc_avg_ms <= ms_per_step
    pipelined_avg_ms = acc_avg_ms
    if not pipelined_ok:
        acc_avg_ms = iso_avg_ms
    alg_bytes = MSM_BYTES_PER_POINT * n  # per launch: one MSM of n points
    achieved_gbs = alg_bytes / (acc_avg_ms * 1e-3) / 1e9 if acc_avg_ms > 0 else 0.0
    glv = n <= (1 << 21)  # BN254 GLV split up to 2^21 points (capi.hip msm_glv_on)
    npts = 2 * n if glv else n                      # virtual points: P_i and phi(P_i)
    c = max(8, min(20, npts.bit_length() - 1 - 4))  # gm choose_window
    windows = -(-128 // c) if glv else -(-255 // c)  # ceil((bits + 1) / c), bits = 127 / 254
    mads = npts * windows * MADS_PER_MIXED_ADD      # ~one XYZZ mixed add per (point, window)
    tmads = mads / (acc_avg_ms * 1e-3) / 1e12 if acc_avg_ms > 0 else 0.0
    traffic = load_pmc_traffic(ACCUM_KERNEL)
    roofline = {
        "kernel": ACCUM_KERNEL + "<Fe<Bn254Fp>> (msm_accum_g1)",
        "bound": "hbm",
        "achieved": round(achieved_gbs, 2),
        "peak": HBM_PEAK_GBS,
        "unit": "GB/s",
        "frac": round(achieved_gbs / HBM_PEAK_GBS, 5),
        "traffic": traffic[0] if traffic else None,
        "traffic_streaming_corrected": traffic[1] if traffic else None,
        "traffic_source": PMC_TRAFFIC_FILE + " (rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes over this MSM "
                          "workload, per launch; traffic = FETCH (64-B gathers are tallied 1:1, calibrated) + WRITE, "
                          "traffic_streaming_corrected = 2 x FETCH + WRITE (the guide's streaming factor); committed "
                          "profile of this kernel, not measured in this run)",
        "avg_launch_ms": round(acc_avg_ms, 4),
        "timing": (("wave stamps of every accumulation launch in the timed loop: the wall clock of its first "
                    "wave's start and last wave's end (csrc/msm_impl.hpp wave_stamp_begin / _end), i.e. the "
                    "kernel's own execution beside the other MSMs' sorts and reductions; the in-flight MSMs' "
                    "accumulations run one after another (gm_ctx::acc_tail).  The launches' "
                    "hipExtLaunchKernelGGL event brackets average %.4f ms: they also hold the time a launch waited "
                    "for wave slots" % bracket_avg_ms) if pipelined_ok and stamped else
                   ("hipExtLaunchKernelGGL start / stop events of every accumulation launch in the timed loop "
                    "(csrc/msm_impl.hpp)") if pipelined_ok else
                   "the timed loop's launch average (%.4f ms) exceeds ms_per_step, so it is not a kernel time: "
                   "avg_launch_ms / achieved / frac are the isolated launch's (below)" % pipelined_avg_ms),
        "timing_source": ("pipelined_wave_stamps" if stamped else "pipelined") if pipelined_ok else "isolated",
        "bytes_per_launch": alg_bytes,
        "int_alu": {"achieved": round(tmads, 3), "peak": round(MAD_PEAK_T, 2), "unit": "T v_mad_u64_u32/s",
                    "frac": round(tmads / MAD_PEAK_T, 4),
                    "work": "%d %spoints x %d windows XYZZ mixed adds x %d mads" % (
                        npts, "GLV (P, phi(P)) " if glv else "", windows, MADS_PER_MIXED_ADD)},
        # the timed steps overlap MSMs (slot streams), so avg_launch_ms above includes
        # the time the accumulation shares the chip with its neighbours' sorts and
        # reductions; the same kernel alone (the synchronous latency MSMs):
        "isolated": ({"avg_launch_ms": round(iso_avg_ms, 4),
                      "achieved": round(alg_bytes / (iso_avg_ms * 1e-3) / 1e9, 2),
                      "frac": round(alg_bytes / (iso_avg_ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 5),
                      "int_alu_frac": round(mads / (iso_avg_ms * 1e-3) / 1e12 / MAD_PEAK_T, 4)}
                     if iso_avg_ms > 0 else None),
        "valu": load_pmc_valu(ACCUM_KERNEL + "<Fe<Bn254Fp> >"),
        "valu_source": PMC_VALU_FILE + " (rocprofv3 --pmc SQ_* passes; committed profile, not measured in this run)",
        "note": "bound=hbm is the bench contract's roofline for this non-MFMA path; the kernel is NOT HBM-bound: "
                "its binding resource is VALU issue -- rocprofv3 PMC (" + PMC_VALU_FILE + ", the 'valu' field) "
                "gives its VALUBusy and VALU instructions per wave (24 entries = 24 mixed adds per thread); "
                "int_alu prices the v_mad_u64_u32 work at the measured mad-only issue peak (DESIGN.md section 3)",
    }
    kernel_ms = {k: round(v[0] / max(v[1], 1), 4) for k, v in stats.items()}

    out = {
        "metric": "BN254 G1 MSM Mpoints/s (2^%d points per GPU, sharded MSM)" % args.logn,
        "value": round(value, 3),
        "unit": "Mpoints/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(ms_per_step, 4),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "u32 limbs (BN254 Fp/Fr Montgomery, integer)",
        "data": "synthetic: uniform scalars, points [k_i]G1 (seeded)",
        "config": {"workload": "BN254 G1 MSM 2^%d random points/scalars per GPU (BASELINE configs[1])" % args.logn,
                   "points_per_gpu": n, "total_points": total_points, "parallelism": "msm-shard%d" % world},
        "roofline": roofline,
        "kernel_avg_ms": kernel_ms,
        "pipeline": ("steps pipelined %d deep (gm_msm_async / gm_msm_wait, one stream per MSM): the next steps' "
                     "device work is queued before step i's host tail (N > 1: incl. the all-gather of partials and "
                     "the host adds); latency_ms = one synchronous (N > 1: sharded) MSM" % PIPE_DEPTH),
        "latency_ms": round(lat_ms, 4),
        "hip_hw_queues": {"value": _process_env("GPU_MAX_HW_QUEUES"),
                          "set_by": "environment" if hwq_preset else "unset (HIP's default)"},
    }

    if rank == 0 and not args.no_secondary and world == 1:
        out["secondary"] = secondary(ctx, gm, args)
    if world > 1 and not args.no_secondary and args.g16_sharded_logn:
        # secondaries must not cost the primary line: a failure is recorded in it
        out["secondary"] = {}
        try:
            g = groth16_sharded_bench(ctx, gm, args.g16_sharded_logn, rank, world, dist, torch)
            out["secondary"]["groth16_sharded"] = g
        except Exception as e:  # noqa: BLE001 -- reported, not hidden
            out["secondary"]["groth16_sharded"] = {"error": repr(e)[:300]}
        # the single-process seam gnark's groth16.Prove uses: rank 0 drives all
        # N GPUs through gm_multi while the other ranks wait at the barrier
        barrier()
        if rank == 0:
            try:
                out["secondary"]["groth16_multi"] = groth16_multi_bench(ctx, gm, args.g16_sharded_logn, world)
            except Exception as e:  # noqa: BLE001
                out["secondary"]["groth16_multi"] = {"error": repr(e)[:300]}
        barrier()
    if rank == 0 and not args.no_cpu_baseline and world == 1:
        out["cpu_baseline"] = cpu_baseline(S, P, n, res)
    if rank == 0:
        print(json.dumps(out))
    ctx.close()
    if dist is not None:
        dist.destroy_process_group()


def _process_env(name):
    """The C environment's value (os.environ does not see a library's setenv)."""
    import ctypes
    libc = ctypes.CDLL(None)
    libc.getenv.restype = ctypes.c_char_p
    v = libc.getenv(name.encode())
    return v.decode() if v else None


R_BN254 = 21888242871839275222246405745257275088548364400416034343698204186575808495617


def add_edge_set(ctx, gm, S, P, n):
    """BASELINE.md §2.2 edge sets inside the config-2 input: 1% of the points at
    infinity ((0,0), every 100th), a run of 1% all-equal points (DummySetup
    shape, setup.go:544-558) and scalars 0, 1, r-1."""
    import numpy as np
    if n < 1024:
        return
    pb = np.frombuffer(P.to_host(), np.uint8).reshape(n, 64).copy()
    pb[::100] = 0
    pb[n // 2:n // 2 + n // 100] = pb[1]
    P.write(pb.tobytes())
    enc = lambda v: (v * (1 << 256) % R_BN254).to_bytes(32, "little")
    S.write(enc(0) + enc(1) + enc(R_BN254 - 1), offset=32 * 7)


def secondary(ctx, gm, args):
    """NTT Gelem/s (config 3) and Groth16 prove time (configs 3/4) on this GPU."""
    res = {}
    nn = 1 << args.ntt_logn
    X = ctx.random_scalars("bn254", nn, 7)
    ctx.ntt("bn254", X, nn, 0, 0, 0)  # builds the domain tables (untimed)
    ctx.ntt("bn254", X, nn, 1, 1, 0)
    ctx.profile_reset()
    ctx.profile(True)
    reps = 5
    t0 = time.perf_counter()
    for _ in range(reps):
        ctx.ntt("bn254", X, nn, 0, 0, 0)   # forward DIF
        ctx.ntt("bn254", X, nn, 1, 1, 0)   # inverse DIT (round trip)
    ctx.synchronize()
    dt = (time.perf_counter() - t0) / (2 * reps)
    ctx.profile(False)
    st = ctx.profile_stats()
    pass_ms, pass_cnt = st.get("ntt_pass", (0.0, 0))
    avg_pass = pass_ms / max(pass_cnt, 1)
    X.free()
    gbs = NTT_BYTES_PER_ELEM * nn / dt / 1e9
    res["ntt"] = {"logn": args.ntt_logn, "gelem_per_s": round(nn / dt / 1e9, 4), "ms_per_transform": round(dt * 1e3, 4),
                  "achieved_gbs": round(gbs, 1), "frac_hbm": round(gbs / HBM_PEAK_GBS, 4),
                  "avg_pass_ms": round(avg_pass, 4), "passes_per_transform": round(pass_cnt / (2 * reps), 2)}
    # the butterflies' products priced at the mad-only issue peak (every radix-2
    # butterfly multiplies once, w^0 included: 162 v_mad_u64_u32 for 9 limbs;
    # inter-pass twiddles, coset / 1/n factors and reductions not counted)
    bfly_mads = args.ntt_logn * (nn // 2) * 2 * 81
    tm = bfly_mads / dt / 1e12
    res["ntt"]["int_alu"] = {"achieved": round(tm, 3), "peak": round(MAD_PEAK_T, 2), "unit": "T v_mad_u64_u32/s",
                             "frac": round(tm / MAD_PEAK_T, 4),
                             "work": "%d stages x %d butterflies x 162 mads" % (args.ntt_logn, nn // 2)}
    if not args.no_cpu_baseline:
        res["ntt"]["cpu_baseline"] = ntt_cpu_baseline(ctx, min(args.ntt_logn, 22))
    if args.msm_extra:
        res["msm"] = {}
        for curve, g2, logn in (("bn254", True, 20), ("bls12377", False, 22), ("bls12377", True, 22)):
            res["msm"]["%s_%s_2^%d" % (curve, "g2" if g2 else "g1", logn)] = msm_line(ctx, gm, curve, g2, logn)
        for curve, g2, logn in (("bn254", False, 20), ("bn254", True, 20)):
            res["msm"]["%s_%s_2^%d_precomputed" % (curve, "g2" if g2 else "g1", logn)] = \
                msm_line(ctx, gm, curve, g2, logn, precompute=True)
    if args.g16_logn:
        plain = [int(l) for l in args.g16_plain.split(",") if l]
        res["groth16"] = []
        for l in (int(x) for x in args.g16_logn.split(",") if x):
            if l in plain:
                # <= 2^20: every scope checked against the oracle, plus the key I/O; the
                # plain 2^24 key: the staged scopes and ONE oracle prove of the host-input
                # proof (its check and the labelled CPU baseline of the headline workload)
                res["groth16"].append(groth16_bench(ctx, gm, l, precompute=False,
                                                    check_oracle=("full" if l <= 20 else
                                                                  "host" if not args.no_cpu_baseline else None),
                                                    staged=True, first_proof=l >= 24))
            if not args.g16_no_precomputed:
                res["groth16"].append(groth16_bench(ctx, gm, l, precompute=True))
            # GM_PK_PRECOMPUTE_AUTO's trade: the window copies' extra upload time
            # against what they save per proof (device inputs)
            ent = {e["pk"]: e for e in res["groth16"] if e["logn"] == l}
            if len(ent) == 2:
                save_ms = ent["plain"]["prove_ms_device_inputs"] - ent["precomputed"]["prove_ms_device_inputs"]
                extra_s = ent["precomputed"]["pk_upload_s"] - ent["plain"]["pk_upload_s"]
                ent["precomputed"]["precompute_break_even"] = {
                    "extra_upload_s": round(extra_s, 3), "saved_ms_per_proof": round(save_ms, 3),
                    "proofs": round(extra_s * 1e3 / save_ms, 1) if save_ms > 0 else None}
    return res


def msm_line(ctx, gm, curve, g2, logn, reps=5, precompute=False):
    """Mpoints/s of one more MSM configuration (BASELINE configs[4]: BLS12-377 G1+G2 2^22).
    precompute: fixed-base window copies prepared once, untimed (a pk / SRS)."""
    n = 1 << logn
    S = ctx.random_scalars(curve, n, 0x5EED0005)
    K = ctx.random_scalars(curve, n, 0x5EED1005)
    P = ctx.batch_mul_base(curve, g2, gm.generator(curve, g2), K, n)
    K.free()
    if precompute:
        pre = ctx.points_upload_precomputed(curve, P.to_host(), g2, 0)
        P.free()
        P = pre
        run = lambda: ctx.msm_precomputed(curve, S, pre, n, g2=g2)
    else:
        run = lambda: ctx.msm(curve, S, P, n, g2=g2)
    run()
    ctx.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        run()
    dt = (time.perf_counter() - t0) / reps
    S.free()
    P.free()
    return {"mpoints_per_s": round(n / dt / 1e6, 3), "ms": round(dt * 1e3, 3)}


def chain_r1cs(ctx, gm, n, nb_wires):
    """Device-resident squaring-chain R1CS with n constraints over nb_wires = n + 2
    wires (one term per matrix and row, coefficient id 1 = one)."""
    import numpy as np
    assert nb_wires == n + 2
    j = np.arange(n - 1, dtype=np.uint32)
    rp = np.arange(n + 1, dtype=np.uint32)
    vl = np.concatenate([2 + j, np.array([0], np.uint32)])
    vr = np.concatenate([2 + j, np.array([n + 1], np.uint32)])
    vo = np.concatenate([3 + j, np.array([1], np.uint32)])
    ones = np.ones(n, np.uint32)
    enc = lambda v: (v * (1 << 256) % R_BN254).to_bytes(32, "little")
    table = b"".join(enc(v) for v in (0, 1, 2, R_BN254 - 1, R_BN254 - 2))
    return gm.R1CS(ctx, "bn254", n, nb_wires, [rp, rp, rp], [ones, ones, ones], [vl, vr, vo], table)


def synthetic_pk(ctx, gm, n, nb_wires, nb_public, slices=None):
    """Synthetic proving key of random points (the DummySetup-style timing key of
    groth16_test.go:70-88; a real setup at 2^24 is out of reach here).  slices:
    {array: (lo, hi)} keeps only those slices (sharded keys)."""
    import numpy as np
    gen1, gen2 = gm.generator("bn254", False), gm.generator("bn254", True)

    def pts(count, g2, seed):
        if count <= 0:
            return np.zeros(0, np.uint8)
        k = ctx.random_scalars("bn254", count, seed)
        p = ctx.batch_mul_base("bn254", g2, gen2 if g2 else gen1, k, count)
        b = np.frombuffer(p.to_host(), np.uint8)
        k.free()
        p.free()
        return b

    cnt = {"g1_A": nb_wires, "g1_B": nb_wires, "g1_Z": n - 1, "g1_K": nb_wires - nb_public, "g2_B": nb_wires}
    sd = {"g1_A": 3, "g1_B": 4, "g1_Z": 5, "g1_K": 6, "g2_B": 7}
    one1 = pts(3, False, 1)
    one2 = pts(2, True, 2)
    pk = {"g1_alpha": one1[:64], "g1_beta": one1[64:128], "g1_delta": one1[128:192],
          "g2_beta": one2[:128], "g2_delta": one2[128:256],
          "infA": np.zeros(nb_wires, np.uint8), "infB": np.zeros(nb_wires, np.uint8)}
    for k, c in cnt.items():
        lo, hi = slices[k] if slices else (0, c)
        pk[k] = pts(hi - lo, k == "g2_B", 1000 * (lo + 1) + sd[k] if slices else sd[k])
    return pk


def groth16_bench(ctx, gm, logn, precompute=True, check_oracle=False, staged=False, first_proof=False):
    """Groth16 prove at n = 2^logn (synthetic pk of random points, synthetic
    solution vectors), timed in two scopes:
      host:   wires / a / b / c in host memory, gm_g16_prove -- the scope of
              icicle.go:204-412 (its H2D copies of a, b, c and wA / wB included);
      device: the same vectors already resident (gm_g16_prove_device).
    check_oracle: "full" -- the timed host-scope and R1CS-resident proofs are
    compared with the oracle prover (prove.go:62-325 restatement) on the same key
    and inputs, plus the staged scopes and the key I/O; "host" -- the staged
    scopes and the host-scope proof only (one oracle prove: the 2^24 headline's
    check and CPU baseline).  staged: the staged scopes also without an oracle
    check (their proofs are compared with the host-scope proof)."""
    import numpy as np
    n = 1 << logn
    nb_wires = n + 2
    nb_public = 2
    pk = synthetic_pk(ctx, gm, n, nb_wires, nb_public)
    ctx.synchronize()
    t0 = time.perf_counter()
    dpk = gm.ProvingKey(ctx, "bn254", pk, n, nb_wires, nb_public, precompute=precompute)
    ctx.synchronize()
    t_upload = time.perf_counter() - t0  # host arrays -> device layout (+ window copies), computeH tables
    W = ctx.random_scalars("bn254", nb_wires, 8)
    srcs = [ctx.random_scalars("bn254", n, 9 + i) for i in range(3)]
    r = ctx.random_scalars("bn254", 2, 12).to_host()
    host = [np.frombuffer(x.to_host(), np.uint8) for x in [W] + srcs]
    A, B, C = (ctx.malloc(32 * n) for _ in range(3))
    # one untimed proof per scope first (arena growth, pinned staging, the
    # R1CS's first touch), then `reps` timed ones: median and best reported
    reps = 3
    t_dev, t_host = [], []
    t_first = None
    for i in range(reps + 1):
        for dst, src in zip((A, B, C), srcs):
            dst.copy_from(src)
        ctx.synchronize()
        t0 = time.perf_counter()
        dpk.prove_device(W, A, B, C, n, r[:32], r[32:])
        if i:
            t_dev.append(time.perf_counter() - t0)
        else:
            t_first = time.perf_counter() - t0  # the key's first prove (its workspace grows)
    # the same after an idle pause as long as the staged scopes' (a gnark prove
    # starts after Solve, with the GPU idle): the GPU's way out of idle costs
    # ~1.3 ms at 2^20 whatever the API (profiles/r06c_staged_overhead.txt)
    t_dev_idle = []
    for i in range(reps):
        for dst, src in zip((A, B, C), srcs):
            dst.copy_from(src)
        ctx.synchronize()
        time.sleep(0.05)
        t0 = time.perf_counter()
        dpk.prove_device(W, A, B, C, n, r[:32], r[32:])
        t_dev_idle.append(time.perf_counter() - t0)
    proof = None
    dpk.prove(host[0], host[1], host[2], host[3], r[:32], r[32:])
    for _ in range(reps):
        ctx.synchronize()
        t0 = time.perf_counter()
        proof = dpk.prove(host[0], host[1], host[2], host[3], r[:32], r[32:])
        t_host.append(time.perf_counter() - t0)
    # R1CS resident (gm_r1cs_upload, once): the squaring chain of
    # groth16_test.go:120-156 over these nb_wires wires (row i: w_{2+i} * w_{2+i}
    # = w_{3+i}, last row 1 * w_{n+1} = Y); per proof only the wires cross PCIe
    ch = chain_r1cs(ctx, gm, n, nb_wires)
    t_r1cs, proof_r1cs = [], None
    dpk.prove_r1cs(ch, host[0], r[:32], r[32:])
    for _ in range(reps):
        ctx.synchronize()
        t0 = time.perf_counter()
        proof_r1cs = dpk.prove_r1cs(ch, host[0], r[:32], r[32:])
        t_r1cs.append(time.perf_counter() - t0)
    # R1CS resident + wires staged during Solve in the reference benchmark
    # circuit's level shape (groth16_test.go:120-156: one solved wire per solver
    # level, solver.go:471-484), gathered as the Go level hook does (a put every
    # 65,536 ids, integration/go/icicle_bn254/staged.go; the replay is the
    # test-only gm_test_stage_replay_chain), then gm_g16_stage_prove_r1cs:
    # nothing crosses PCIe after Solve
    t_r1cs_staged, proof_r1cs_staged, ns_level = [], None, []
    for i in range(reps + 1):
        st = dpk.stage(n)
        ns_level.append(st.replay_chain(host[0], 3, n))
        ctx.synchronize()
        time.sleep(0.05)  # the staged copies finish during "Solve"
        t0 = time.perf_counter()
        proof_r1cs_staged = st.prove_r1cs(ch, r[:32], r[32:])
        if i:
            t_r1cs_staged.append(time.perf_counter() - t0)
        st.free()
    ch.free()
    med = lambda v: sorted(v)[len(v) // 2]
    res = {"logn": logn, "pk": "precomputed" if precompute else "plain",
           "roofline": groth16_roofline(n, nb_wires, precompute, med(t_dev)),
           "prove_ms_host_inputs": round(med(t_host) * 1e3, 3), "prove_ms_device_inputs": round(med(t_dev) * 1e3, 3),
           "prove_ms_device_inputs_after_idle": round(med(t_dev_idle) * 1e3, 3),
           "prove_ms_r1cs_resident": round(med(t_r1cs) * 1e3, 3),
           "prove_ms_r1cs_resident_wires_staged": round(med(t_r1cs_staged) * 1e3, 3),
           "r1cs_staged_matches_r1cs_resident": bool(proof_r1cs_staged == proof_r1cs),
           "best_ms": {"host_inputs": round(min(t_host) * 1e3, 3), "device_inputs": round(min(t_dev) * 1e3, 3),
                       "r1cs_resident": round(min(t_r1cs) * 1e3, 3),
                       "r1cs_resident_wires_staged": round(min(t_r1cs_staged) * 1e3, 3)},
           "pk_upload_s": round(t_upload, 3), "first_prove_ms_device_inputs": round(t_first * 1e3, 3),
           "stage_host_ns_per_level_wires": round(sorted(ns_level)[len(ns_level) // 2], 1),
           "runs": reps, "warmup": 1, "stat": "median",
           "scope": "host_inputs = icicle.go:204-412 incl. H2D of wires/a/b/c; device_inputs = same with inputs "
                    "resident; r1cs_resident = host wires only (a/b/c from the device-resident R1CS, "
                    "gm_g16_prove_r1cs); r1cs_resident_wires_staged = the same with the wires staged during "
                    "Solve in one-wire solver levels (gm_g16_stage_prove_r1cs, the Go default path with the "
                    "wire level hook; stage_host_ns_per_level_wires = the Solve-side cost of that staging); all "
                    "after Solve; device_inputs_after_idle and the staged scopes start after a 50 ms idle "
                    "pause (Solve), the other scopes right after GPU work; pk_upload_s = host arrays to the device key incl. window copies and computeH "
                    "tables; first_prove_ms_device_inputs = the key's first prove in this process"}
    if check_oracle or staged:
        res.update(staged_bench(ctx, dpk, n, host, r, proof))
    if check_oracle == "full":
        res.update(io_bench(ctx, gm, dpk, pk, n, nb_wires, nb_public, host, r, proof))
    dpk.free()
    if first_proof:
        res["time_to_first_proof"] = first_proof_bench(gm, pk, n, nb_wires, nb_public, host, r, proof)
    for b in [W, A, B, C] + srcs:
        b.free()
    if check_oracle:
        sys.path.insert(0, os.path.join(ROOT, "oracle"))
        import oracle_lib
        threads, model = host_cpu()
        pk["sizes"] = np.array([n, nb_wires, nb_wires, nb_wires, nb_wires - nb_public], np.uint64)
        t0 = time.perf_counter()
        exp = oracle_lib.g16_prove("bn254", pk, nb_public, host[0], host[1], host[2], host[3], r[:32], r[32:],
                                   nthreads=threads)
        cpu_s = time.perf_counter() - t0
        res["matches_oracle"] = bool(exp == proof)
        if check_oracle == "full":
            # the R1CS-resident proof: a, b, c of the chain from the same wires
            wv = host[0].reshape(nb_wires, 32)
            ca = np.concatenate([wv[2:n + 1], wv[0:1]])
            cb = np.concatenate([wv[2:n + 1], wv[n + 1:n + 2]])
            cc = np.concatenate([wv[3:n + 2], wv[1:2]])
            exp_r1cs = oracle_lib.g16_prove("bn254", pk, nb_public, host[0], ca.tobytes(), cb.tobytes(),
                                            cc.tobytes(), r[:32], r[32:], nthreads=threads)
            res["r1cs_resident_matches_oracle"] = bool(exp_r1cs == proof_r1cs)
        # the labelled CPU baseline of this workload (BASELINE.md §2.1 asks for
        # groth16_bn254.Prove beside the GPU; no Go on the box -> the port)
        res["cpu_baseline"] = {
            "value": round(cpu_s * 1e3, 1), "unit": "ms per proof", "cores": threads, "kind": "port",
            "cpu_model": model,
            "sample": "one full 2^%d Groth16 prove on the same key and inputs (computeH + 4 G1 + 1 G2 "
                      "signed-digit Pippenger MSMs + finishing adds): oracle/gm_oracle.cpp restatement of "
                      "prove.go:62-325, not gnark-crypto (no Go toolchain on the box)" % logn,
            "gpu_over_cpu": round(cpu_s * 1e3 / max(res["prove_ms_host_inputs"], 1e-9), 1)}
    return res


def _choose_window(n, bits=254):
    """msm_impl.hpp choose_window: c in [8, 20] minimising n W + 3 W 2^(c-1)."""
    best = None
    for c in range(8, 21):
        W = -(-(bits + 1) // c)
        cost = n * W + 3 * W * (1 << (c - 1))
        if best is None or cost < best[0]:
            best = (cost, c, W)
    return best[1], best[2]


def _choose_precomp(n, bits=254):
    """msm_sort.hip msm_choose_precomp: c in [8, 24] minimising n W + 3 2^(c-1)."""
    best = None
    for c in range(8, 25):
        W = -(-(bits + 1) // c)
        cost = n * W + 3 * (1 << (c - 1))
        if best is None or cost < best[0]:
            best = (cost, c, W)
    return best[1], best[2]


# v_mad_u64_u32 per lazily reduced XYZZ mixed add (ISA counts of the
# accumulation loops, tools/isa_blocks.py): BN254 G1 one lane; BN254 G2 both
# lanes of a lane pair (pair_fp2.hpp, four-product Y3)
MADS_G1_ADD = MADS_PER_MIXED_ADD
MADS_G2_ADD = 2 * 1701  # per lane: 1296 + 405 in the k_msm_accum_seg_pair loop blocks


def groth16_roofline(n, nb_wires, precompute, t_s):
    """Roofline of one Groth16 prove at n = 2^logn (device inputs, the kernels'
    own time scope): SURVEY §8d's algorithmic bytes (1120 B per domain element)
    over the prove time against HBM, and the summed MSM bucket-add mads over the
    prove time against the measured mad-only peak (int_alu)."""
    choose = _choose_precomp if precompute else _choose_window
    _, W = choose(nb_wires)      # A, B, B2, K: the shared wire plan over the wires
    _, Wz = choose(n - 1)        # Z over h[:n-1]
    g1_adds = 3 * nb_wires * W + (n - 1) * Wz
    g2_adds = nb_wires * W
    mads = g1_adds * MADS_G1_ADD + g2_adds * MADS_G2_ADD
    nbytes = G16_BYTES_PER_ELEM * n
    gbs = nbytes / t_s / 1e9
    tm = mads / t_s / 1e12
    return {"bound": "hbm", "achieved": round(gbs, 2), "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": round(gbs / HBM_PEAK_GBS, 5), "bytes_per_prove": nbytes, "traffic": None,
            "basis": "SURVEY.md 8d: 4 x 96 n (G1 MSMs) + 160 n (G2 MSM) + 7 x 64 n (NTTs) + 128 n (PolyOps) "
                     "over prove_ms_device_inputs",
            "int_alu": {"achieved": round(tm, 3), "peak": round(MAD_PEAK_T, 2), "unit": "T v_mad_u64_u32/s",
                        "frac": round(tm / MAD_PEAK_T, 4),
                        "work": "%d G1 + %d G2 mixed adds (W = %d, Wz = %d windows%s) x %d / %d mads; NTTs and "
                                "reductions not counted" % (g1_adds, g2_adds, W, Wz,
                                                             ", precomputed" if precompute else "",
                                                             MADS_G1_ADD, MADS_G2_ADD)}}


def staged_bench(ctx, dpk, n, host, r, host_proof):
    """SURVEY.md §8f row 4 on the same key (gm_g16_stage_*): a / b / c and the
    wires handed over during "Solve" in the reference benchmark circuit's level
    shape (groth16_test.go:120-156, a chain of squarings: every solver level
    finishes one constraint and solves one wire, solver.go:471-484), gathered as
    the Go level hook does (integration/go/icicle_bn254/staged.go: a put every
    65,536 ids; replayed by the test-only gm_test_stage_replay_chain), then only
    the prove timed (gm_g16_stage_prove).  The first stage is an untimed warm-up
    (the key keeps the stage buffers for the next proof).  The Solve-side cost
    per level is reported for the gathered puts and, on a 2^20-level sample, for
    one put per level and vector (no gathering in the hook)."""
    out = {}
    reps = 3
    ts, ns, proof = [], [], None
    abc = (host[1], host[2], host[3])
    for i in range(reps + 1):
        st = dpk.stage(n)
        ns.append(st.replay_chain(host[0], 3, n, abc=abc))
        ctx.synchronize()
        time.sleep(0.05)  # the staged copies finish during "Solve"
        t0 = time.perf_counter()
        proof = st.prove(r[:32], r[32:])
        if i:
            ts.append(time.perf_counter() - t0)
        st.free()
    k = min(n, 1 << 20)
    st = dpk.stage(n)
    ns_each = st.replay_chain(host[0], 3, k, abc=abc, coalesce=False)
    st.free()
    out["prove_ms_staged_all_during_solve"] = round(sorted(ts)[reps // 2] * 1e3, 3)
    out["staged_matches_host_scope"] = bool(proof == host_proof)
    out["stage_host_ns_per_level"] = {"gathered": round(sorted(ns)[len(ns) // 2], 1),
                                      "one_put_per_level_and_vector": round(ns_each, 1),
                                      "levels": n, "sample_levels_one_put": k}
    out["staged_scope"] = ("a/b/c and wires staged during Solve in one-constraint / one-wire levels (gathered "
                           "puts, as staged.go's hook), prove only timed")
    return out


def io_bench(ctx, gm, dpk, pk, n, nb_wires, nb_public, host, r, proof):
    """SURVEY.md §8f row 3 on the same key:
      dump:   the key's five point arrays written as WriteDump slices
              (marshal.go:389-456) to a local file, then streamed into device
              buffers (gm_g16_pk_upload_dump) -- file read + H2D + conversion;
      cache:  save / load of the device-layout key (gm_g16_pk_save_cache / load)."""
    import tempfile
    out = {}
    meta = {k: pk[k] for k in ("g1_alpha", "g1_beta", "g1_delta", "g2_beta", "g2_delta", "infA", "infB")}
    meta["counts"] = (nb_wires, nb_wires, nb_wires - nb_public)
    with tempfile.TemporaryDirectory() as d:
        path = os.path.join(d, "pk.dump")
        off = gm.write_dump_slices(path, "bn254", pk, b"\0" * 4096)
        nbytes = os.path.getsize(path) - off
        t0 = time.perf_counter()
        k2, _ = gm.ProvingKey.from_dump(ctx, "bn254", path, off, meta, n, nb_wires, nb_public)
        t_dump = time.perf_counter() - t0
        ok = k2.prove(host[0], host[1], host[2], host[3], r[:32], r[32:]) == proof
        cpath = os.path.join(d, "pk.cache")
        t0 = time.perf_counter()
        k2.save_cache(cpath)
        t_save = time.perf_counter() - t0
        t0 = time.perf_counter()
        k3 = gm.ProvingKey.from_cache(ctx, cpath, like=k2)
        t_load = time.perf_counter() - t0
        ok = ok and k3.prove(host[0], host[1], host[2], host[3], r[:32], r[32:]) == proof
        k2.free()
        k3.free()
    out["pk_dump"] = {"bytes": nbytes, "upload_s": round(t_dump, 4), "gb_per_s": round(nbytes / t_dump / 1e9, 2),
                      "cache_save_s": round(t_save, 4), "cache_load_s": round(t_load, 4),
                      "proofs_match": bool(ok),
                      "note": "dump file in the page cache (local tmp); device-layout cache = same point bytes"}
    return out


def first_proof_bench(gm, pk, n, nb_wires, nb_public, host, r, proof):
    """Time to first proof (the reference uploads the key
    lazily inside the first Prove, icicle.go:145-150 -> :31-130): the key written
    as a WriteDump file (marshal.go:389-456), then in a FRESH process each
    (tools/first_proof.py): library + context, the key streamed from the dump
    (plain / GM_PK_PRECOMPUTE_AUTO, which picks the window copies on MI355X) or
    read back from a device-layout cache of the plain key, and the first and a
    second host-input prove.  Files in the local TMPDIR."""
    import subprocess
    import tempfile
    out = {}
    meta = {k: pk[k] for k in ("g1_alpha", "g1_beta", "g1_delta", "g2_beta", "g2_delta", "infA", "infB")}
    meta["counts"] = (nb_wires, nb_wires, nb_wires - nb_public)
    with tempfile.TemporaryDirectory() as d:
        path = os.path.join(d, "pk.dump")
        t0 = time.perf_counter()
        off = gm.write_dump_slices(path, "bn254", pk, b"\0" * 4096)
        out["dump_bytes"] = os.path.getsize(path) - off
        out["dump_write_s"] = round(time.perf_counter() - t0, 2)
        inp = os.path.join(d, "inputs.npz")
        np_ = __import__("numpy")
        np_.savez(inp, **{k: np_.asarray(v) for k, v in meta.items() if k != "counts"},
                  counts=np_.array(meta["counts"], np_.uint64), domain_size=n, nb_wires=nb_wires,
                  nb_public=nb_public, W=host[0], a=host[1], b=host[2], c=host[3], r=np_.frombuffer(r, np_.uint8))

        def child(target, mode):
            t = time.perf_counter()
            rr = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "first_proof.py"), inp, target, str(off),
                                 mode], capture_output=True, text=True, timeout=600)
            if rr.returncode != 0:
                return {"error": (rr.stderr or rr.stdout)[-300:]}
            j = json.loads(rr.stdout.strip().splitlines()[-1])
            j["process_wall_s"] = round(time.perf_counter() - t, 3)
            j["proof_matches"] = bytes.fromhex(j.pop("proof_hex")) == b"".join(proof)
            return j

        out["fresh_process_dump_plain"] = child(path, "0")
        out["fresh_process_dump_auto"] = child(path, "auto")
        # the device-layout cache of the plain key, written by a key streamed from the dump
        cpath = os.path.join(d, "pk.cache")
        import gnark_mi355x as gmm
        ctx2 = gmm.Context(0)
        try:
            k2, _ = gmm.ProvingKey.from_dump(ctx2, "bn254", path, off, meta, n, nb_wires, nb_public)
            t0 = time.perf_counter()
            k2.save_cache(cpath)
            out["cache_save_s"] = round(time.perf_counter() - t0, 2)
            k2.free()
        finally:
            ctx2.close()
        os.remove(path)
        out["fresh_process_cache_plain"] = child(cpath, "cache")
    out["note"] = ("fresh process per line (python + numpy + the library, no torch); to_first_proof_s counts from "
                   "the interpreter's first statement; dump / cache files in the local TMPDIR (page cache)")
    return out


def groth16_sharded_bench(ctx, gm, logn, rank, world, dist, torch):
    """BASELINE config 4: Groth16 prove at n = 2^logn with the G1/G2 MSMs sharded
    across the ranks (one GPU each).  Every rank holds only its slice of each pk
    point array (synthetic random points, precomputed) and the replicated solved
    vectors; computeH runs on every rank, the five partial MSM sums are
    all-gathered over RCCL and finished on the host (gnark_mi355x.sharded_prove).
    Timed with barriers + device syncs on both sides, max over ranks."""
    n = 1 << logn
    nb_wires = n + 2
    nb_public = 2
    gen1, gen2 = gm.generator("bn254", False), gm.generator("bn254", True)

    def pts(count, g2, seed):
        import numpy as np
        if count == 0:
            return np.zeros(0, np.uint8)
        k = ctx.random_scalars("bn254", count, seed)
        p = ctx.batch_mul_base("bn254", g2, gen2 if g2 else gen1, k, count)
        b = p.to_host()
        k.free()
        p.free()
        return np.frombuffer(b, np.uint8)

    import numpy as np
    one1 = pts(3, False, 1)
    one2 = pts(2, True, 2)
    nbA = nbB = nb_wires
    nbK = nb_wires - nb_public

    def sl(count):
        lo, hi = gm.shard_range(count, world, rank)
        return hi - lo

    sd = 1000 * (rank + 1)
    pk = {"g1_alpha": one1[:64], "g1_beta": one1[64:128], "g1_delta": one1[128:192],
          "g1_A": pts(sl(nbA), False, sd + 3), "g1_B": pts(sl(nbB), False, sd + 4),
          "g1_Z": pts(sl(n - 1), False, sd + 5), "g1_K": pts(sl(nbK), False, sd + 6),
          "g2_beta": one2[:128], "g2_delta": one2[128:256], "g2_B": pts(sl(nbB), True, sd + 7),
          "infA": np.zeros(nb_wires, np.uint8), "infB": np.zeros(nb_wires, np.uint8),
          "shard_sizes": (nbA, nbB, nbK)}
    dpk = gm.ProvingKey(ctx, "bn254", pk, n, nb_wires, nb_public, precompute=True, shard=(rank, world),
                        pk_is_shard=True)
    W = ctx.random_scalars("bn254", nb_wires, 8)
    A, B, C = (ctx.malloc(32 * n) for _ in range(3))
    srcs = [ctx.random_scalars("bn254", n, 9 + i) for i in range(3)]
    r = ctx.random_scalars("bn254", 2, 12).to_host()
    times = []
    for _ in range(2):
        for dst, src in zip((A, B, C), srcs):
            dst.copy_from(src)
        ctx.synchronize()
        dist.barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        gm.sharded_prove(dpk, W, A, B, C, n, r[:32], r[32:])
        ctx.synchronize()
        dist.barrier()
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        tt = torch.tensor([dt], dtype=torch.float64, device="cuda" if dist.get_backend() == "nccl" else "cpu")
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        times.append(float(tt.item()))
    dpk.free()
    for b in [W, A, B, C] + srcs:
        b.free()
    return {"logn": logn, "n_gpus": world, "prove_ms": round(min(times) * 1e3, 3), "pk": "precomputed, sharded",
            "note": "computeH replicated per rank; 5 MSMs sharded; partials all-gathered over RCCL; after Solve"}


def host_cpu():
    """(threads this process may use, CPU model string)."""
    try:
        cores = len(os.sched_getaffinity(0))
    except AttributeError:
        cores = os.cpu_count() or 1
    # the GPU box grants a CPU share through a cgroup quota while affinity and
    # nproc show the whole machine: more threads than the quota only contend
    quota = None
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, per = f.read().split()[:2]
            if q != "max":
                quota = max(1, int(int(q) / int(per)))
    except (OSError, ValueError):
        pass
    if quota is None and os.environ.get("OMP_NUM_THREADS", "").isdigit():
        quota = int(os.environ["OMP_NUM_THREADS"])
    if quota:
        cores = min(cores, quota)
    model = "unknown"
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    model = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    return cores, model


def groth16_multi_bench(ctx, gm, logn, ndev, precompute=True):
    """BASELINE config 4 through the single-process multi-device C-ABI
    (gm_g16_prove_multi): one host thread per GPU, key sharded across GPUs
    0..ndev-1, wire slices / a, b, c to device 0 / h slices over xGMI, host
    inputs (icicle.go:204-412 scope incl. H2D)."""
    import numpy as np
    n = 1 << logn
    nb_wires, nb_public = n + 2, 2
    pk = synthetic_pk(ctx, gm, n, nb_wires, nb_public)
    vecs = [ctx.random_scalars("bn254", m, 8 + i) for i, m in enumerate((nb_wires, n, n, n))]
    host = [np.frombuffer(v.to_host(), np.uint8) for v in vecs]
    for v in vecs:
        v.free()
    r = ctx.random_scalars("bn254", 2, 12).to_host()
    nvis = gm.device_count()  # < ndev only in the one-GPU gloo rehearsal
    with gm.Multi([d % nvis for d in range(ndev)]) as m:
        t0 = time.perf_counter()
        mpk = gm.ProvingKeyMulti(m, "bn254", pk, n, nb_wires, nb_public, precompute=precompute)
        t_up = time.perf_counter() - t0
        times = []
        for _ in range(3):
            t0 = time.perf_counter()
            mpk.prove(host[0], host[1], host[2], host[3], r[:32], r[32:])
            times.append(time.perf_counter() - t0)
        mpk.free()
    return {"logn": logn, "n_gpus": ndev, "prove_ms_host_inputs": round(sorted(times)[1] * 1e3, 3), "runs": 3,
            "stat": "median", "pk_upload_s": round(t_up, 2), "pk": "precomputed" if precompute else "plain",
            "note": "one process, one host thread per GPU (gm_multi); computeH on GPU 0, h slices peer-copied"}


def ntt_cpu_baseline(ctx, logn):
    """Oracle radix-2 FFT (fft.Domain.FFT restatement, oracle/gm_oracle.cpp) on the
    box's CPU share: forward DIF + inverse DIT of a 2^logn vector (bounded
    sample; the GPU line is 2^24)."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle_lib
    threads, model = host_cpu()
    n = 1 << logn
    X = ctx.random_scalars("bn254", n, 7)
    xb = X.to_host()
    X.free()
    t0 = time.perf_counter()
    y = oracle_lib.fft("bn254", xb, False, False, False, nthreads=threads)
    z = oracle_lib.fft("bn254", y, True, True, False, nthreads=threads)
    dt = (time.perf_counter() - t0) / 2
    return {"value": round(n / dt / 1e9, 4), "unit": "Gelem/s", "cores": threads, "kind": "port", "cpu_model": model,
            "sample": "2^%d BN254 Fr FFT + FFTInverse round trip (oracle restatement of fft.Domain, not "
                      "gnark-crypto)" % logn, "round_trip_ok": bool(z == xb)}


def cpu_baseline(S, P, n, gpu_jac):
    """Oracle C++ Pippenger (the 'port') on the host cores this process may use
    (the box's CPU share), same 2^logn workload incl. the edge set, checked
    against the GPU result."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle_lib
    threads, model = host_cpu()
    sb, pb = S.to_host(), P.to_host()
    oracle_lib.msm("bn254", False, sb[: 32 * 1024], pb[: 64 * 1024], nthreads=threads)  # warm
    t0 = time.perf_counter()
    reps = 0
    while True:
        aff = oracle_lib.msm("bn254", False, sb, pb, nthreads=threads)
        reps += 1
        if time.perf_counter() - t0 > 10 or reps >= 3:
            break
    dt = (time.perf_counter() - t0) / reps
    import gnark_mi355x as gm
    match = gm.jac_to_affine("bn254", False, gpu_jac) == aff
    return {"value": round(n / dt / 1e6, 4), "unit": "Mpoints/s", "cores": threads, "kind": "port",
            "cpu_model": model,
            "sample": "full 2^%d-point BN254 G1 MSM (same input, edge set incl.), %d rep(s), C++ signed-digit "
                      "XYZZ-bucket Pippenger (gnark-crypto MultiExp's shape, oracle/), not gnark-crypto (no Go "
                      "toolchain on the box)"
                      % (n.bit_length() - 1, reps),
            "result_matches_gpu": bool(match)}


if __name__ == "__main__":
    main()
