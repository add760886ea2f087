/*
 * gnark_mi355x.h -- C-ABI of the MI355X (gfx950) MSM + NTT backend for gnark's
 * Groth16 prover.  Drop-in replacement for the device layer that
 * backend/groth16/bn254/icicle/icicle.go binds through
 * github.com/ingonyama-zk/iciclegnark v0.1.0 (go.mod:15; not vendored -- the
 * signatures below are the ones its call sites in icicle.go imply).
 *
 * Conventions
 *  - Plain C, no torch / HIP types in signatures.  Device buffers are opaque
 *    `void*` device pointers owned by the caller and released with gm_free
 *    (iciclegnark's unsafe.Pointer + FreeDevicePointer model).
 *  - Host pointers are only read/written during the call and never retained
 *    (cgo rule).  Every entry point selects its context's device itself.
 *  - Memory layout is gnark-crypto's, byte for byte: fr.Element / fp.Element =
 *    little-endian u64 limbs in Montgomery form; G1Affine {X,Y}; G2Affine
 *    {X.A0,X.A1,Y.A0,Y.A1}; G1Jac/G2Jac {X,Y,Z}; infinity affine = all zero.
 *  - Every function returns GM_OK (0) or a negative gm_status; the message of
 *    the last failure on the calling thread is available from gm_last_error().
 *  - Calls on one context are serialised; use one context per thread/GPU for
 *    concurrency.  Multi-GPU: either one process drives every GPU through one
 *    gm_multi handle: gm_g16_pk_upload_multi / gm_g16_prove_multi, or one process per
 *    GPU holds a key shard (gm_g16_pk_upload_shard / gm_g16_prove_partial).
 */
#ifndef GNARK_MI355X_H
#define GNARK_MI355X_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef enum {
  GM_OK = 0,
  GM_ERR_INVALID = -1,     /* bad argument / unsupported size */
  GM_ERR_DEVICE = -2,      /* HIP runtime error */
  GM_ERR_OOM = -3,         /* device allocation failed */
  GM_ERR_UNSUPPORTED = -4, /* curve/group combination not built */
} gm_status;

typedef enum { GM_BN254 = 0, GM_BLS12_377 = 1 } gm_curve;

typedef struct gm_ctx gm_ctx;

/* ---- context ---------------------------------------------------------- */
const char* gm_last_error(void);
int gm_version(void);
/* Number of visible HIP devices. */
int gm_device_count(int* count);
/* Creates a context on HIP device `device` with its own streams. */
int gm_init(int device, gm_ctx** out);
int gm_destroy(gm_ctx* ctx);
int gm_synchronize(gm_ctx* ctx);
/* Releases the device memory a context keeps for reuse between calls: the
 * workspace arenas, the a / b / c input buffer of host-input proves (3 n Fr,
 * 1.5 GB at 2^24), the pinned H2D ring, the cached NTT domain tables and the
 * staging buffers parked with keys by gm_g16_stage_free (3 n + nb_wires Fr plus
 * 64 MiB pinned and 64 MiB device per key).  All
 * are re-created on demand by the next call that needs them.  Refused
 * (GM_ERR_INVALID) while gm_msm_async MSMs are pending.  Call it before
 * uploading a key whose GM_PK_PRECOMPUTE_AUTO decision should see that memory
 * as free. */
int gm_trim(gm_ctx* ctx);
/* Per-kernel timing with HIP events on the context stream (bench/profiling). */
int gm_profile_enable(gm_ctx* ctx, int on);
int gm_profile_reset(gm_ctx* ctx);
/* Fetches accumulated time (ms) and launch count for kernel `name`. */
int gm_profile_get(gm_ctx* ctx, const char* name, double* total_ms, uint64_t* count);
/* Writes "name total_ms count\n" lines into buf (truncated to cap). */
int gm_profile_dump(gm_ctx* ctx, char* buf, size_t cap);
/* Test/tuning knob: force the MSM window size c (0 = automatic). */
int gm_set_msm_window(gm_ctx* ctx, int c);
/* GLV split (k = k1 + k2 lambda over P_i and phi(P_i), BN254 and BLS12-377) of
 * MSMs over gnark-layout points: mode 1 on, 0 off, -1 default (on up to 2^21
 * points unless GM_MSM_GLV=0; G2 also unless GM_MSM_GLV_G2=0).  Tuning / A-B
 * knob; results are identical either way. */
int gm_set_msm_glv(gm_ctx* ctx, int mode);

/* ---- memory (iciclegnark CopyToDevice / CopyPointsToDevice /
 *      CopyG2PointsToDevice / FreeDevicePointer; icicle.go:44,47,65,90,95,
 *      109,114,125,245,269,352,356,416-418,478-480,492,505-507) ---------- */
int gm_malloc(gm_ctx* ctx, size_t bytes, void** dev_out);
int gm_free(gm_ctx* ctx, void* dev);
int gm_copy_to_device(gm_ctx* ctx, const void* host, size_t bytes, void** dev_out);
int gm_memcpy_h2d(gm_ctx* ctx, void* dev, const void* host, size_t bytes);
int gm_memcpy_d2h(gm_ctx* ctx, void* host, const void* dev, size_t bytes);
int gm_memcpy_d2d(gm_ctx* ctx, void* dst_dev, const void* src_dev, size_t bytes);
/* Uploads n gnark affine points of (curve, g2) -> device buffer. */
int gm_copy_points_to_device(gm_ctx* ctx, int curve, int g2, const void* host_points, size_t n,
                             void** dev_out);

/* ---- MSM (iciclegnark MsmOnDevice icicle.go:302,315,332,355 and
 *      MsmG2OnDevice icicle.go:382; CPU twin G1Jac/G2Jac.MultiExp
 *      prove.go:204,217,237,247,293) ------------------------------------
 * out = sum_i int(scalars[i]) * points[i], scalars = n Montgomery fr.Element,
 * points = n gnark affine points ((0,0) = infinity is allowed), both resident
 * on the device.  out_jac receives gnark's G1Jac (3 x fp) / G2Jac (3 x E2)
 * layout; out_affine (optional, may be NULL) receives the affine form. */
int gm_msm(gm_ctx* ctx, int curve, int g2, const void* scalars_dev, const void* points_dev,
           size_t n, void* out_jac, void* out_affine);
/* Pipelined MSM: gm_msm_async queues the device work of gm_msm (same
 * arguments) and returns at once; gm_msm_wait finishes it (host tail: checks
 * and the Horner combination) and frees the handle.  The host tail of one MSM
 * thus overlaps the device work of the next one issued before it.  At most three
 * MSMs may be in flight per context; wait in issue order.  Each in-flight MSM
 * runs on a stream of its own (GM_MSM_SLOT_STREAMS=0: the context stream), at
 * the highest stream priority (a hardware-queue pool of their own, so they do
 * not share a queue with the context's other streams; GM_MSM_SLOT_PRIO=0: normal
 * priority), so one MSM's reduction overlaps the next one's conversion and sort.
 * The MSM starts after the work already queued on the context stream (its
 * inputs).  gm_msm_async and gm_msm_wait queue nothing on the context stream;
 * the next call that does waits there for the pending MSMs' input reads first.
 * (The library also raises GPU_MAX_HW_QUEUES to 8 at load time when the
 * variable is unset.)  Synchronous calls
 * (gm_msm, gm_msm_prepared, gm_ntt, ...) may be made on the same context while
 * async MSMs are pending: each pending MSM keeps its own scratch arena and its
 * own pinned readback buffer until its gm_msm_wait, and work queued on the
 * context after gm_msm_async returns starts only once that MSM has read its
 * scalars and points, so such a call may overwrite them in place.
 * gm_destroy with MSMs pending waits for their device work and releases their
 * resources; each pending handle stays allocated, and its gm_msm_wait returns
 * GM_ERR_INVALID ("context was destroyed") and frees it. */
typedef struct gm_msm_pending gm_msm_pending;
int gm_msm_async(gm_ctx* ctx, int curve, int g2, const void* scalars_dev, const void* points_dev, size_t n,
                 gm_msm_pending** out);
int gm_msm_wait(gm_msm_pending* pending, void* out_jacobian, void* out_affine);
/* gm_msm with the scalars in host memory (copied on the context stream). */
int gm_msm_host_scalars(gm_ctx* ctx, int curve, int g2, const void* scalars_host,
                        const void* points_dev, size_t n, void* out_jac, void* out_affine);

/* Device-resident point sets (a proving key's arrays, a KZG SRS): upload n gnark
 * affine points once, converted to the MSM's internal layout (same byte size),
 * and run MSMs over any prefix of them without per-call conversion.  Free with
 * gm_free.  (setupDevicePointers, icicle.go:90-125, keeps pk points resident.) */
int gm_points_upload(gm_ctx* ctx, int curve, int g2, const void* host_points, size_t n,
                     void** prepared_out);
int gm_msm_prepared(gm_ctx* ctx, int curve, int g2, const void* scalars_dev, const void* prepared,
                    size_t n, void* out_jac, void* out_affine);

/* Fixed-base precomputation (ICICLE's MSM precompute_factor idea, re-derived):
 * besides the n points, W-1 copies [2^(c w)] P_i (w = 1..W-1) are stored, so
 * every window's digits share one bucket set and the bucket reduction runs
 * once instead of W times (and c can grow).  window = c in [2, 24], or 0 =
 * automatic from n.  Memory: W x the plain prepared size.  The copy count W =
 * ceil((r_bits + 1) / c) is reported by gm_precompute_layout.  An MSM over
 * any prefix n <= prepared_n of the set passes the SAME prepared_n and window
 * used at upload. */
int gm_precompute_layout(int curve, size_t prepared_n, int window, int* c_out, int* copies_out);
int gm_points_upload_precomputed(gm_ctx* ctx, int curve, int g2, const void* host_points, size_t n,
                                 int window, void** prepared_out);
int gm_msm_precomputed(gm_ctx* ctx, int curve, int g2, const void* scalars_dev, const void* prepared,
                       size_t prepared_n, int window, size_t n, void* out_jac, void* out_affine);

/* ---- KZG commitment (PLONK; backend/plonk/bls12-377/prove.go:312,460,718,
 *      1158-1168 call gnark-crypto kzg.Commit) ---------------------------------
 * digest = sum_i coeffs[i] * srs[i] over the first n points of a prepared SRS
 * (pk.Kzg.G1 or pk.KzgLagrange.G1, setup.go:81-82), coeffs = n Montgomery
 * fr.Elements in host memory.  GM_ERR_INVALID if n > srs_len (kzg.ErrInvalidPolynomialSize). */
int gm_kzg_commit(gm_ctx* ctx, int curve, const void* srs_prepared, size_t srs_len,
                  const void* coeffs_host, size_t n, void* digest_affine);

/* ---- NTT (iciclegnark GenerateTwiddleFactors icicle.go:68,73;
 *      INttOnDevice :489,502; NttOnDevice :490; PolyOps :500;
 *      ReverseScalars :510; CPU twin fft.Domain.FFT/FFTInverse
 *      prove.go:372-378,396) ---------------------------------------------
 * In-place transform of n = 2^k Montgomery fr.Elements with gnark-crypto
 * fft.Domain semantics:
 *   inverse = 0: coefficients -> evaluations at w^i (g*w^i if coset)
 *   inverse = 1: evaluations -> coefficients, scaled by 1/n (and g^-i if coset)
 *   dit = 0 (DIF): natural-order input, bit-reversed output
 *   dit = 1 (DIT): bit-reversed input, natural-order output
 * w = the domain generator of fft.NewDomain(n), g = FrMultiplicativeGen
 * (5 for BN254, 22 for BLS12-377). */
int gm_ntt(gm_ctx* ctx, int curve, void* data_dev, size_t n, int inverse, int dit, int coset);
/* a[i] <- (a[i]*b[i] - c[i]) * den   (PolyOps, den = (g^n - 1)^-1 broadcast) */
int gm_poly_ops(gm_ctx* ctx, int curve, void* a_dev, const void* b_dev, const void* c_dev,
                size_t n, const void* den_host);
/* In-place bit-reversal permutation of n = 2^k Fr elements (ReverseScalars). */
int gm_reverse_scalars(gm_ctx* ctx, int curve, void* data_dev, size_t n);

/* ---- iciclegnark call-for-call binding (icicle.go:68-76,489-510) --------
 * Same buffer ownership and element order as iciclegnark v0.1.0, so a cgo shim
 * can bind INttOnDevice / NttOnDevice / PolyOps / GenerateTwiddleFactors name
 * for name and icicle.go's computeH (icicle.go:453-513) runs unchanged,
 * including its FreeDevicePointer calls:
 *  - gm_icicle_intt_on_device: natural-order evaluations at in_dev -> a NEW
 *    device buffer (*out_dev, free with gm_free) of natural-order coefficients
 *    (times g^-i / n on the coset); in_dev is left bit-reversed, as iciclegnark
 *    leaves it (INttOnDevice, icicle.go:489,502).
 *  - gm_icicle_ntt_on_device: natural-order coefficients at in_dev -> natural-
 *    order evaluations (on the coset g*w^i if coset) at out_dev (NttOnDevice,
 *    icicle.go:490); out_dev == in_dev is allowed.
 *  - gm_icicle_poly_ops: a[i] <- (a[i]*b[i] - c[i]) * den[i], den a device
 *    vector (PolyOps with pk.DenDevice, icicle.go:52-65,500).
 *  - gm_icicle_generate_twiddles: builds the context's cached domain of size n
 *    and returns a freeable device token for pk.DomainDevice.Twiddles(Inv)
 *    (GenerateTwiddleFactors, icicle.go:68,73).
 * ReverseScalars (icicle.go:510) is gm_reverse_scalars, MsmOnDevice /
 * MsmG2OnDevice are gm_msm, CopyToDevice / CopyPointsToDevice are
 * gm_copy_to_device / gm_copy_points_to_device, FreeDevicePointer is gm_free. */
int gm_icicle_generate_twiddles(gm_ctx* ctx, int curve, size_t n, int inverse, void** token_out);
int gm_icicle_intt_on_device(gm_ctx* ctx, int curve, void* in_dev, size_t n, int coset, void** out_dev);
int gm_icicle_ntt_on_device(gm_ctx* ctx, int curve, void* out_dev, const void* in_dev, size_t n, int coset);
int gm_icicle_poly_ops(gm_ctx* ctx, int curve, void* a_dev, const void* b_dev, const void* c_dev,
                       const void* den_dev, size_t n);

/* ---- Groth16 computeH (icicle.go:453-513; prove.go:356-399) -----------
 * a, b, c: `len` Montgomery fr.Elements each (the R1CS solution vectors),
 * device-resident, zero-padded in place to n = domain size (buffers must hold
 * n elements).  On return a_dev holds h in BIT-REVERSED coefficient order
 * (matching pk.G1.Z, setup.go:265-267); b_dev and c_dev are clobbered. */
int gm_groth16_compute_h(gm_ctx* ctx, int curve, void* a_dev, void* b_dev, void* c_dev,
                         size_t len, size_t n);

/* ---- Groth16 prover (icicle_bn254.Prove, icicle.go:133-422; CPU twin
 *      groth16_bn254.Prove prove.go:62-325, without the BSB22 commitment
 *      side path) ---------------------------------------------------------
 * A proving key whose point arrays live on the device (uploaded once, as
 * icicle's setupDevicePointers, icicle.go:31-130). */
typedef struct gm_g16_pk gm_g16_pk;
typedef struct {
  size_t domain_size;      /* n = pk.Domain.Cardinality */
  size_t nb_wires;         /* len(InfinityA) */
  size_t nb_public;        /* r1cs.GetNbPublicVariables() (incl. ONE wire) */
  size_t nbA, nbB, nbK;    /* len(pk.G1.A), len(pk.G1.B), len(pk.G1.K) */
  const void* g1_alpha;    /* G1Affine */
  const void* g1_beta;
  const void* g1_delta;
  const void* g1_A;        /* nbA points */
  const void* g1_B;        /* nbB points */
  const void* g1_Z;        /* n-1 points, bit-reversed (setup.go:265-267) */
  const void* g1_K;        /* nbK points */
  const void* g2_beta;     /* G2Affine */
  const void* g2_delta;
  const void* g2_B;        /* nbB points */
  const uint8_t* infA;     /* nb_wires flags (InfinityA) */
  const uint8_t* infB;     /* nb_wires flags (InfinityB) */
  /* nbK wire indices whose values multiply pk.G1.K: wireValues[nb_public:]
   * minus the private-committed and commitment wires (prove.go:243-245,
   * filterHeap :331-354).  NULL = no commitments: nb_public + i. */
  const uint32_t* k_wires;
} gm_g16_pk_host;

int gm_g16_pk_upload(gm_ctx* ctx, int curve, const gm_g16_pk_host* pk, gm_g16_pk** out);
/* flags: GM_PK_PRECOMPUTE keeps fixed-base window copies of every point array
 * on the device (gm_points_upload_precomputed; ~12x the point memory at 2^24,
 * ~77 GB for a BN254 2^24 key) -- fewer windows and one bucket reduction per
 * MSM.  gm_g16_pk_upload(...) == gm_g16_pk_upload_ex(..., 0, ...). */
#define GM_PK_PRECOMPUTE 1u
/* GM_PK_PRECOMPUTE_AUTO: precompute when the window copies fit the device --
 * the key's precomputed arrays plus the upload's transient buffers take at
 * most GM_PK_PRECOMPUTE_FRAC (default 0.6) of the free device memory at upload
 * time (hipMemGetInfo); otherwise a plain key.  On a 288 GB MI355X a BN254
 * 2^24 key (~77 GB precomputed) qualifies.  gm_g16_pk_precomputed() reports
 * the choice. */
#define GM_PK_PRECOMPUTE_AUTO 2u
int gm_g16_pk_precomputed(const gm_g16_pk* pk, int* out);
int gm_g16_pk_upload_ex(gm_ctx* ctx, int curve, const gm_g16_pk_host* pk, unsigned flags, gm_g16_pk** out);
int gm_g16_pk_free(gm_ctx* ctx, gm_g16_pk* pk);

/* Proves with solved vectors in host memory: wires (nb_wires Fr), a, b, c
 * (nb_constraints Fr each), r and s (one Fr each, Montgomery).  Outputs
 * proof.Ar (G1Affine), proof.Bs (G2Affine), proof.Krs (G1Affine).  The wires
 * are copied first; a, b, c are copied on a separate stream by a helper thread
 * while the A/B/K MSMs run (the icicle.go:204-412 scope, H2D included). */
int gm_g16_prove(gm_ctx* ctx, gm_g16_pk* pk, const void* wires, const void* a, const void* b,
                 const void* c, size_t nb_constraints, const void* r, const void* s,
                 void* ar_out, void* bs_out, void* krs_out);
/* Same with wires/a/b/c already resident on the device (a, b, c buffers hold
 * n elements and are clobbered). */
int gm_g16_prove_device(gm_ctx* ctx, gm_g16_pk* pk, const void* wires_dev, void* a_dev,
                        void* b_dev, void* c_dev, size_t nb_constraints, const void* r,
                        const void* s, void* ar_out, void* bs_out, void* krs_out);

/* ---- R1CS resident on the device: a proof from the wires alone ------------
 * gnark's solver produces solution.A/B/C as <L_i, w>, <R_i, w>, <O_i, w>
 * (constraint/bn254/solver.go:540-620); with the constraint system on the
 * device (uploaded once, like the key) only the wires cross PCIe per proof.
 * Per matrix m in {L, R, O}: rowptr[m] (nb_constraints + 1 entries, from 0),
 * cid[m] / vid[m] (rowptr[m][nb_constraints] terms: coefficient id into
 * `coeffs`, wire id, or GM_R1CS_CONST for a constant term -- constraint.Term,
 * constraint/term.go:31-40); coeffs = the CoeffTable (coeff.go:30-44,
 * ncoeffs fr.Element, Montgomery; ids 0 and 1 must be zero and one).  Ids are
 * validated at upload. */
#define GM_R1CS_CONST 0xFFFFFFFFu
typedef struct gm_r1cs gm_r1cs;
int gm_r1cs_upload(gm_ctx* ctx, int curve, size_t nb_constraints, size_t nb_wires, const uint32_t* const* rowptr,
                   const uint32_t* const* cid, const uint32_t* const* vid, const void* coeffs, size_t ncoeffs,
                   gm_r1cs** out);
int gm_r1cs_free(gm_ctx* ctx, gm_r1cs* r1cs);
/* a_dev, b_dev, c_dev (nb_constraints Fr each) from device-resident wires. */
int gm_r1cs_eval(gm_ctx* ctx, const gm_r1cs* r1cs, const void* wires_dev, void* a_dev, void* b_dev, void* c_dev);
/* gm_g16_prove with the wires as the only host input: wires copied, a / b / c
 * evaluated on the device ahead of computeH while the MSMs run.  The key must
 * be whole (not a shard) and match the constraint system. */
int gm_g16_prove_r1cs(gm_ctx* ctx, gm_g16_pk* pk, const gm_r1cs* r1cs, const void* wires, const void* r,
                      const void* s, void* ar_out, void* bs_out, void* krs_out);

/* ---- sharded Groth16 (BASELINE config 4: G1/G2 MSMs split across the GPUs of
 *      a node, one process per GPU) -------------------------
 * Rank `rank` of `world` uploads only its contiguous slice [lo, hi) of each
 * point array (lo/hi as gnark_mi355x.shard_range: the first n % world ranks
 * hold one extra point) of pk.G1.A (nbA), pk.G1.B and pk.G2.B (nbB), pk.G1.K
 * (nbK) and pk.G1.Z (n - 1).  In `pk` the counts nbA/nbB/nbK and the flags
 * infA/infB/k_wires describe the WHOLE key, while g1_A, g1_B, g1_K, g1_Z and
 * g2_B point at the first point of this rank's slice.  world = 1 is
 * gm_g16_pk_upload_ex. */
int gm_g16_pk_upload_shard(gm_ctx* ctx, int curve, const gm_g16_pk_host* pk, unsigned flags, int rank,
                           int world, gm_g16_pk** out);
/* Size of one partial: 4 G1Jac (sums over A, B, K, Z) + 1 G2Jac (B2). */
int gm_g16_partial_bytes(int curve, size_t* out);
/* computeH over the whole domain (every rank holds the solved a, b, c and the
 * wires), then the five MSMs over this rank's slices: writes the raw sums
 * [sum_A, sum_B, sum_K, sum_Z] (G1Jac) and sum_B2 (G2Jac), no blinding. */
int gm_g16_prove_partial(gm_ctx* ctx, gm_g16_pk* pk, const void* wires_dev, void* a_dev, void* b_dev,
                         void* c_dev, size_t nb_constraints, void* partial_out);
/* Host only: proof elements from the rank-summed partials (same layout) with
 * the blinding of icicle.go:295-391 (alpha, beta, [r]delta, [s]delta,
 * [-rs]delta, [s]Ar, [r]Bs1, [s]delta2, beta2 from `pk`). */
int gm_g16_finish(int curve, const gm_g16_pk_host* pk, const void* sums, const void* r, const void* s,
                  void* ar_out, void* bs_out, void* krs_out);

/* ---- single-process multi-device Groth16 (one gnark process drives every
 *      GPU of the node behind unchanged groth16.Prove call sites,
 *      backend/groth16/groth16.go:192-204) ---------------
 * gm_multi_init creates one context (own streams) per entry of device_ids
 * (entries may repeat: several contexts on one GPU rehearse the multi-GPU path).
 * gm_g16_pk_upload_multi shards every point array of the key across the
 * devices (device 0, which also runs computeH, takes a smaller share:
 * GM_MULTI_SHARE0, default 0.6 of the others'); each device keeps only the
 * compaction-map slices of its shard and later receives only the wires those
 * slices read.  gm_g16_prove_multi runs one host thread per device: wires
 * slices to every device, a / b / c to device 0 (computeH there, h slices sent
 * to the other devices by peer copies over xGMI), the five partial MSMs
 * everywhere, then host adds of the per-device sums and the finishing of
 * gm_g16_finish.  Output and inputs as gm_g16_prove. */
typedef struct gm_multi gm_multi;
typedef struct gm_g16_pk_multi gm_g16_pk_multi;
int gm_multi_init(const int* device_ids, int count, gm_multi** out);
int gm_multi_destroy(gm_multi* m);
int gm_multi_size(const gm_multi* m, int* count);
int gm_multi_context(gm_multi* m, int index, gm_ctx** out);
int gm_g16_pk_upload_multi(gm_multi* m, int curve, const gm_g16_pk_host* pk, unsigned flags,
                           gm_g16_pk_multi** out);
int gm_g16_pk_free_multi(gm_multi* m, gm_g16_pk_multi* pk);
int gm_g16_prove_multi(gm_multi* m, gm_g16_pk_multi* pk, const void* wires, const void* a, const void* b,
                       const void* c, size_t nb_constraints, const void* r, const void* s, void* ar_out,
                       void* bs_out, void* krs_out);

/* ---- proving-key I/O --------------------------------
 * gnark's ProvingKey.WriteDump (backend/groth16/bn254/marshal.go:389-456)
 * writes, after its header (unsafe marker, Domain, the raw-encoded alpha /
 * beta / delta, nbWires, NbInfinityA/B, InfinityA/B, nbCommitments), the five
 * point slices G1.A, G1.B, G1.Z, G1.K, G2.B with gnark-crypto's
 * utils/unsafe.WriteSlice: a little-endian uint64 element count followed by
 * the raw G1Affine / G2Affine memory -- this ABI's point layout.
 * gm_g16_pk_upload_dump reads those five slices from `fd` starting at byte
 * `offset` (where ReadDump, marshal.go:511, starts reading them) and streams
 * them into device buffers (pread into pinned buffers; H2D and conversion /
 * GM_PK_PRECOMPUTE precomputation per 64 MiB chunk, overlapped with the
 * reads).  `meta` carries the header fields as in gm_g16_pk_upload; its point
 * pointers are ignored and its nbA / nbB / nbK (and domain_size - 1 for G1.Z)
 * must equal the slice lengths in the file.  *end_offset receives the first
 * byte after G2.B (the commitment keys' slices, marshal.go:532-543, follow).
 * The _shard form reads only rank's slice of every array (as
 * gm_g16_pk_upload_shard).  The file position of fd is not used or moved. */
int gm_g16_pk_upload_dump(gm_ctx* ctx, int curve, const gm_g16_pk_host* meta, int fd, uint64_t offset,
                          unsigned flags, uint64_t* end_offset, gm_g16_pk** out);
int gm_g16_pk_upload_dump_shard(gm_ctx* ctx, int curve, const gm_g16_pk_host* meta, int fd, uint64_t offset,
                                unsigned flags, int rank, int world, uint64_t* end_offset, gm_g16_pk** out);
/* A device-resident key (shard) in its device layout, GM_PK_PRECOMPUTE window
 * copies included, written to `fd` at its current position; load_cache reads
 * one back with no conversion or precomputation (the persisted device form of
 * SURVEY.md §5's checkpoint row). */
int gm_g16_pk_save_cache(gm_ctx* ctx, const gm_g16_pk* pk, int fd);
int gm_g16_pk_load_cache(gm_ctx* ctx, int fd, gm_g16_pk** out);

/* ---- staged prover inputs --------------------------
 * The R1CS solver (constraint/bn254/solver.go:426-532) makes a, b, c final
 * level by level.  Each level (or range) can be handed over as soon as it is
 * solved: every put copies its host data into a pinned ring before it returns
 * (no host pointer is kept) and queues the copy to the device on the
 * context's copy stream, so the H2D overlaps the rest of Solve.
 * gm_g16_stage_prove waits for the queued copies and proves from the
 * device-resident inputs (gm_g16_prove_device).  Every element of a, b, c
 * [0, nb_constraints) and of the wires [0, nb_wires) must have been put; the
 * prove consumes a, b, c (one proof per stage).  gm_g16_stage_free keeps the
 * stage's device vectors and pinned ring with the key (one spare per key,
 * released by gm_g16_pk_free), and the next gm_g16_stage_begin on the same
 * context reuses them: no allocation per proof (GM_G16_STAGE_REUSE=0: off).
 * Indexed puts are gathered as records (element id, vector, value) in the open
 * ring slot and queued when it holds 65,536 of them, when it is full, before a
 * range put and before the prove: a put of one element (a solver level that
 * solved one wire) costs its 40-byte record, not a copy and a launch. */
typedef struct gm_g16_stage gm_g16_stage;
#define GM_STAGE_A 0
#define GM_STAGE_B 1
#define GM_STAGE_C 2
#define GM_STAGE_WIRES 3
int gm_g16_stage_begin(gm_ctx* ctx, gm_g16_pk* pk, size_t nb_constraints, gm_g16_stage** out);
/* elements [lo, lo + count) of vector `which`; host_src points at element lo */
int gm_g16_stage_put_range(gm_g16_stage* st, int which, size_t lo, size_t count, const void* host_src);
/* elements idx[0..k) of vector `which` (one solver level), read from host_base[idx[j]] */
int gm_g16_stage_put_indexed(gm_g16_stage* st, int which, const void* host_base, const uint32_t* idx, size_t k);
int gm_g16_stage_prove(gm_g16_stage* st, const void* r, const void* s, void* ar_out, void* bs_out,
                       void* krs_out);
/* The wires-only staged proof of a resident constraint system: the wires were
 * put during Solve (GM_STAGE_WIRES, e.g. per solver level), a, b, c come from
 * the device R1CS (gm_r1cs_upload) -- nothing crosses PCIe after Solve.  The
 * stage's a / b / c need not be put (they receive the evaluation). */
int gm_g16_stage_prove_r1cs(gm_g16_stage* st, const gm_r1cs* r1cs, const void* r, const void* s, void* ar_out,
                            void* bs_out, void* krs_out);
int gm_g16_stage_free(gm_g16_stage* st);

/* ---- host-side group helpers (finishing adds of sharded MSMs) ---------- */
/* out = p + q, all gnark Jacobian (G1Jac or G2Jac). */
int gm_jac_add(int curve, int g2, const void* p, const void* q, void* out);
/* affine_out = p in affine form. */
int gm_jac_to_affine(int curve, int g2, const void* p, void* affine_out);

/* ---- synthetic inputs (bench / tests; not on the hot path) ------------
 * out[i] = [k_i] base, k_i = Montgomery fr.Elements on the device, outputs
 * affine points on the device (curve.BatchScalarMultiplicationG1/G2). */
int gm_batch_mul_base(gm_ctx* ctx, int curve, int g2, const void* base_affine_host,
                      const void* scalars_dev, size_t n, void* points_out_dev);
/* Fills n Montgomery Fr elements uniform in [0, r) from a seed (device). */
int gm_random_scalars(gm_ctx* ctx, int curve, uint64_t seed, size_t n, void* scalars_dev);
/* Generator points of the curve in gnark affine layout (host). */
int gm_generator(int curve, int g2, void* affine_out);

/* Element-wise test hooks of the device field / curve layer live in a separate
 * test-only library (include/gnark_mi355x_testhooks.h,
 * libgnark_mi355x_testhooks.so); the product library does not export them. */

#ifdef __cplusplus
}
#endif
#endif /* GNARK_MI355X_H */
