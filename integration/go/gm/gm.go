//go:build icicle

// Package gm is the cgo binding of libgnark_mi355x (include/gnark_mi355x.h)
// shared by the gnark hooks in this directory (icicle_bn254, icicle_bls12377,
// plonk_bls12377) and by the iciclegnark-compatible shim
// (iciclegnark/curves/bn254).
//
// NOT COMPILED HERE: this image has no Go toolchain.  The C side it binds is
// built and tested by the repo (tests/test_capi_symbols.py, tests/*_gpu.py).
//
// Devices: GNARK_MI355X_DEVICES="0,1,..." selects the GPUs one process drives
// (default: every visible device).  With more than one, Groth16 keys are
// sharded across them (gm_g16_pk_upload_multi) and proofs run on all of them
// from the one gnark process (gm_g16_prove_multi) -- groth16.Prove's call
// sites (backend/groth16/groth16.go:192-204) stay unchanged.
package gm

/*
#cgo CFLAGS: -I${SRCDIR}/../../../include
#cgo LDFLAGS: -L${SRCDIR}/../../../gnark-icicle_amd -lgnark_mi355x -Wl,-rpath,${SRCDIR}/../../../gnark-icicle_amd
#include <stdlib.h>
#include "gnark_mi355x.h"
*/
import "C"

import (
	"errors"
	"fmt"
	"os"
	"runtime"
	"strconv"
	"strings"
	"sync"
	"unsafe"
)

// Curve ids of the C-ABI.
const (
	BN254     = C.GM_BN254
	BLS12_377 = C.GM_BLS12_377
)

// PkPrecompute keeps fixed-base window copies of every proving-key point array
// on the device(s) (GM_PK_PRECOMPUTE).
const PkPrecompute = C.GM_PK_PRECOMPUTE

// PkPrecomputeAuto takes the window copies only when they fit the device
// (GM_PK_PRECOMPUTE_AUTO: at most 60% of the free HBM at upload; a BN254 2^24
// key needs ~77 GB of an MI355X's 288 GB).
const PkPrecomputeAuto = C.GM_PK_PRECOMPUTE_AUTO

// PrecomputeFlags maps GNARK_MI355X_PRECOMPUTE to upload flags: "1" always,
// "auto" when the copies fit (PkPrecomputeAuto), unset or "0" never.  The
// copies pay off only for a key that proves many times: at 2^24 (BN254, one
// MI355X) they add 4.3 s to the upload and save 9.8 ms per proof, break-even
// ~440 proofs; at 2^20 0.28 s against 1.3 ms, ~220 proofs (bench.py
// precompute_break_even, profiles/r06e_bench.json).  A process that proves once
// reaches its first proof in 3.1 s plain against 7.1 s precomputed.
func PrecomputeFlags() uint {
	switch os.Getenv("GNARK_MI355X_PRECOMPUTE") {
	case "1":
		return PkPrecompute
	case "auto":
		return PkPrecomputeAuto
	default:
		return 0
	}
}

func lastErr(what string, rc C.int) error {
	return fmt.Errorf("gnark_mi355x %s: status %d: %s", what, int(rc), C.GoString(C.gm_last_error()))
}

var (
	once    sync.Once
	devices []C.int
	ctx0    *C.gm_ctx  // context on devices[0]: MSM / NTT / KZG calls
	multi   *C.gm_multi // all devices (nil when only one)
	initErr error
)

func initDevices() {
	var n C.int
	if rc := C.gm_device_count(&n); rc != C.GM_OK {
		initErr = lastErr("gm_device_count", rc)
		return
	}
	if s := os.Getenv("GNARK_MI355X_DEVICES"); s != "" {
		for _, f := range strings.Split(s, ",") {
			d, err := strconv.Atoi(strings.TrimSpace(f))
			if err != nil {
				initErr = fmt.Errorf("GNARK_MI355X_DEVICES: %w", err)
				return
			}
			devices = append(devices, C.int(d))
		}
	} else {
		for d := C.int(0); d < n; d++ {
			devices = append(devices, d)
		}
	}
	if len(devices) == 0 {
		initErr = errors.New("gnark_mi355x: no GPU visible")
		return
	}
	if rc := C.gm_init(devices[0], &ctx0); rc != C.GM_OK {
		initErr = lastErr("gm_init", rc)
		return
	}
	if len(devices) > 1 {
		if rc := C.gm_multi_init(&devices[0], C.int(len(devices)), &multi); rc != C.GM_OK {
			initErr = lastErr("gm_multi_init", rc)
		}
	}
}

// Ctx returns the context of the first selected device.
func Ctx() (*C.gm_ctx, error) {
	once.Do(initDevices)
	return ctx0, initErr
}

// NbDevices is the number of GPUs this process proves on.
func NbDevices() int {
	once.Do(initDevices)
	return len(devices)
}

// ---------------------------------------------------------------------------
// Groth16
// ---------------------------------------------------------------------------

// G16HostKey mirrors gm_g16_pk_host: the gnark proving-key arrays, passed by
// pointer (gnark-crypto's G1Affine / G2Affine / fr.Element layouts are the
// C-ABI's), read only during the upload.
type G16HostKey struct {
	DomainSize, NbWires, NbPublic uint64
	NbA, NbB, NbK                 uint64
	Alpha, Beta, Delta            unsafe.Pointer // *G1Affine
	A, B, Z, K                    unsafe.Pointer // first element of each []G1Affine
	Beta2, Delta2                 unsafe.Pointer // *G2Affine
	B2                            unsafe.Pointer // first element of []G2Affine
	InfA, InfB                    []bool         // pk.InfinityA / InfinityB
	KWires                        []uint32       // nil, or the filterHeap survivors (prove.go:243-245)
}

// G16Key is a proving key resident on the GPU(s) (setupDevicePointers,
// icicle.go:31-130).
type G16Key struct {
	curve  C.int
	single *C.gm_g16_pk
	multi  *C.gm_g16_pk_multi
}

func boolsToBytes(b []bool) []byte {
	out := make([]byte, len(b))
	for i, v := range b {
		if v {
			out[i] = 1
		}
	}
	return out
}

// cHost fills the C-ABI's gm_g16_pk_host from k.  cgo rule: &h is a Go pointer
// handed to C, so every Go pointer stored IN h must be pinned for the call
// (runtime.Pinner, Go >= 1.21; the reference pins Go 1.22, go.mod:3) -- without
// it the default GODEBUG=cgocheck=1 panics with "cgo argument has Go pointer to
// unpinned Go pointer".  The caller unpins after the C call returns; the library
// never keeps these pointers (include/gnark_mi355x.h).  withPoints=false leaves
// the point-array fields nil (the dump upload reads them from the file).
func (k *G16HostKey) cHost(pin *runtime.Pinner, withPoints bool) C.gm_g16_pk_host {
	pinned := func(p unsafe.Pointer) unsafe.Pointer {
		if p != nil {
			pin.Pin(p)
		}
		return p
	}
	h := C.gm_g16_pk_host{
		domain_size: C.size_t(k.DomainSize), nb_wires: C.size_t(k.NbWires), nb_public: C.size_t(k.NbPublic),
		nbA: C.size_t(k.NbA), nbB: C.size_t(k.NbB), nbK: C.size_t(k.NbK),
		g1_alpha: pinned(k.Alpha), g1_beta: pinned(k.Beta), g1_delta: pinned(k.Delta),
		g2_beta: pinned(k.Beta2), g2_delta: pinned(k.Delta2),
	}
	if withPoints {
		h.g1_A, h.g1_B, h.g1_Z, h.g1_K = pinned(k.A), pinned(k.B), pinned(k.Z), pinned(k.K)
		h.g2_B = pinned(k.B2)
	}
	if len(k.InfA) > 0 {
		infA := boolsToBytes(k.InfA)
		h.infA = (*C.uint8_t)(pinned(unsafe.Pointer(&infA[0])))
	}
	if len(k.InfB) > 0 {
		infB := boolsToBytes(k.InfB)
		h.infB = (*C.uint8_t)(pinned(unsafe.Pointer(&infB[0])))
	}
	if len(k.KWires) > 0 {
		h.k_wires = (*C.uint32_t)(pinned(unsafe.Pointer(&k.KWires[0])))
	}
	return h
}

// UploadG16Key uploads k once (sharded across the GPUs when there are several).
func UploadG16Key(curve int, k *G16HostKey, flags uint) (*G16Key, error) {
	ctx, err := Ctx()
	if err != nil {
		return nil, err
	}
	var pin runtime.Pinner
	defer pin.Unpin()
	h := k.cHost(&pin, true)
	key := &G16Key{curve: C.int(curve)}
	if multi != nil {
		if rc := C.gm_g16_pk_upload_multi(multi, C.int(curve), &h, C.uint(flags), &key.multi); rc != C.GM_OK {
			return nil, lastErr("gm_g16_pk_upload_multi", rc)
		}
	} else if rc := C.gm_g16_pk_upload_ex(ctx, C.int(curve), &h, C.uint(flags), &key.single); rc != C.GM_OK {
		return nil, lastErr("gm_g16_pk_upload_ex", rc)
	}
	return key, nil
}

// Free releases the device copies.
func (k *G16Key) Free() {
	if k.multi != nil {
		C.gm_g16_pk_free_multi(multi, k.multi)
	}
	if k.single != nil {
		C.gm_g16_pk_free(ctx0, k.single)
	}
}

// Prove runs the device part of the Groth16 prover (icicle.go:204-412 /
// prove.go:140-313): computeH, the compaction, the five MSMs and the finishing
// adds.  wires, a, b, c point at the first fr.Element of solution.W, .A, .B,
// .C; r, s at the sampled fr.Elements; ar, krs at G1Affine and bs at G2Affine.
func (k *G16Key) Prove(wires, a, b, c unsafe.Pointer, nbConstraints int, r, s, ar, bs, krs unsafe.Pointer) error {
	if k.multi != nil {
		if rc := C.gm_g16_prove_multi(multi, k.multi, wires, a, b, c, C.size_t(nbConstraints), r, s, ar, bs, krs); rc != C.GM_OK {
			return lastErr("gm_g16_prove_multi", rc)
		}
		return nil
	}
	if rc := C.gm_g16_prove(ctx0, k.single, wires, a, b, c, C.size_t(nbConstraints), r, s, ar, bs, krs); rc != C.GM_OK {
		return lastErr("gm_g16_prove", rc)
	}
	return nil
}

// R1CS is a constraint system resident on device 0 (gm_r1cs_upload): proofs then
// need the wires alone (ProveR1CS), a / b / c are evaluated on the GPU.
type R1CS struct{ h *C.gm_r1cs }

// R1CSConst marks a constant term's wire id (constraint.Term.IsConstant).
const R1CSConst = C.GM_R1CS_CONST

// UploadR1CS uploads the CSR form of r1cs.GetR1Cs() (per matrix L, R, O: row
// pointers, coefficient ids, wire ids) and the CoeffTable (coeffs points at
// the first fr.Element of r1cs.Coefficients).
func UploadR1CS(curve int, nbConstraints, nbWires int, rowptr, cid, vid [3][]uint32, coeffs unsafe.Pointer,
	ncoeffs int) (*R1CS, error) {
	ctx, err := Ctx()
	if err != nil {
		return nil, err
	}
	// the three pointer arrays live in C memory: a Go array of Go pointers
	// would itself need every element pinned (§2.1 of INTEGRATION.md)
	arr := func(v [3][]uint32) **C.uint32_t {
		p := (*[3]*C.uint32_t)(C.malloc(C.size_t(3 * unsafe.Sizeof(uintptr(0)))))
		for m := 0; m < 3; m++ {
			p[m] = nil
			if len(v[m]) > 0 {
				p[m] = (*C.uint32_t)(unsafe.Pointer(&v[m][0]))
			}
		}
		return &p[0]
	}
	var pin runtime.Pinner
	defer pin.Unpin()
	for m := 0; m < 3; m++ {
		for _, v := range [][]uint32{rowptr[m], cid[m], vid[m]} {
			if len(v) > 0 {
				pin.Pin(&v[0])
			}
		}
	}
	rp, ci, vi := arr(rowptr), arr(cid), arr(vid)
	defer C.free(unsafe.Pointer(rp))
	defer C.free(unsafe.Pointer(ci))
	defer C.free(unsafe.Pointer(vi))
	r := &R1CS{}
	if rc := C.gm_r1cs_upload(ctx, C.int(curve), C.size_t(nbConstraints), C.size_t(nbWires), rp, ci, vi, coeffs,
		C.size_t(ncoeffs), &r.h); rc != C.GM_OK {
		return nil, lastErr("gm_r1cs_upload", rc)
	}
	return r, nil
}

// Free releases the device copy.
func (r *R1CS) Free() { C.gm_r1cs_free(ctx0, r.h) }

// ProveR1CS is Prove with the wires as the only host input (single-device keys).
func (k *G16Key) ProveR1CS(r1 *R1CS, wires unsafe.Pointer, r, s, ar, bs, krs unsafe.Pointer) error {
	if k.single == nil {
		return errors.New("gnark_mi355x: ProveR1CS needs a single-device key")
	}
	if rc := C.gm_g16_prove_r1cs(ctx0, k.single, r1.h, wires, r, s, ar, bs, krs); rc != C.GM_OK {
		return lastErr("gm_g16_prove_r1cs", rc)
	}
	return nil
}

// UploadG16KeyDump streams the five point slices of a WriteDump file
// (marshal.go:389-456) from f, starting at byte offset (where ReadDump,
// marshal.go:511, starts reading them), straight into device buffers; k holds
// the header fields (its point pointers are ignored).  Returns the offset just
// past G2.B (the commitment keys' slices follow).  With several GPUs every
// device streams its own shard of each array (gm_g16_pk_upload_dump_shard);
// proofs then run per device and are summed on the host like UploadG16Key's.
func UploadG16KeyDump(curve int, k *G16HostKey, f *os.File, offset int64, flags uint) (*G16Key, int64, error) {
	ctx, err := Ctx()
	if err != nil {
		return nil, 0, err
	}
	if multi != nil {
		return nil, 0, errors.New("gnark_mi355x: dump streaming drives one device; use UploadG16Key with several")
	}
	var pin runtime.Pinner
	defer pin.Unpin()
	h := k.cHost(&pin, false) // the point arrays come from the file
	key := &G16Key{curve: C.int(curve)}
	var end C.uint64_t
	if rc := C.gm_g16_pk_upload_dump(ctx, C.int(curve), &h, C.int(f.Fd()), C.uint64_t(offset), C.uint(flags), &end,
		&key.single); rc != C.GM_OK {
		return nil, 0, lastErr("gm_g16_pk_upload_dump", rc)
	}
	return key, int64(end), nil
}

// SaveCache writes the device copy of k (with its precomputed window copies)
// to f in the device layout; LoadG16KeyCache reads it back with no conversion
// or precomputation.
func (k *G16Key) SaveCache(f *os.File) error {
	if k.single == nil {
		return errors.New("gnark_mi355x: SaveCache needs a single-device key")
	}
	if rc := C.gm_g16_pk_save_cache(ctx0, k.single, C.int(f.Fd())); rc != C.GM_OK {
		return lastErr("gm_g16_pk_save_cache", rc)
	}
	return nil
}

func LoadG16KeyCache(curve int, f *os.File) (*G16Key, error) {
	ctx, err := Ctx()
	if err != nil {
		return nil, err
	}
	key := &G16Key{curve: C.int(curve)}
	if rc := C.gm_g16_pk_load_cache(ctx, C.int(f.Fd()), &key.single); rc != C.GM_OK {
		return nil, lastErr("gm_g16_pk_load_cache", rc)
	}
	return key, nil
}

// Vectors of a staged proof (gm_g16_stage_*).
const (
	StageA     = C.GM_STAGE_A
	StageB     = C.GM_STAGE_B
	StageC     = C.GM_STAGE_C
	StageWires = C.GM_STAGE_WIRES
)

// G16Stage collects a, b, c (and the wires) while the solver runs.
type G16Stage struct{ h *C.gm_g16_stage }

// Stage starts a staged proof of nbConstraints constraints (single device).
func (k *G16Key) Stage(nbConstraints int) (*G16Stage, error) {
	if k.single == nil {
		return nil, errors.New("gnark_mi355x: staged inputs need a single-device key")
	}
	st := &G16Stage{}
	if rc := C.gm_g16_stage_begin(ctx0, k.single, C.size_t(nbConstraints), &st.h); rc != C.GM_OK {
		return nil, lastErr("gm_g16_stage_begin", rc)
	}
	return st, nil
}

// PutIndexed hands over base[idx[j]] of vector which (one solver level).
func (st *G16Stage) PutIndexed(which int, base unsafe.Pointer, idx []uint32) error {
	if len(idx) == 0 {
		return nil
	}
	if rc := C.gm_g16_stage_put_indexed(st.h, C.int(which), base, (*C.uint32_t)(unsafe.Pointer(&idx[0])),
		C.size_t(len(idx))); rc != C.GM_OK {
		return lastErr("gm_g16_stage_put_indexed", rc)
	}
	return nil
}

// PutRange hands over elements [lo, lo+n) of vector which; src points at element lo.
func (st *G16Stage) PutRange(which int, lo, n int, src unsafe.Pointer) error {
	if rc := C.gm_g16_stage_put_range(st.h, C.int(which), C.size_t(lo), C.size_t(n), src); rc != C.GM_OK {
		return lastErr("gm_g16_stage_put_range", rc)
	}
	return nil
}

// Prove waits for the staged copies and proves (Ar, Bs, Krs as G16Key.Prove).
func (st *G16Stage) Prove(r, s, ar, bs, krs unsafe.Pointer) error {
	if rc := C.gm_g16_stage_prove(st.h, r, s, ar, bs, krs); rc != C.GM_OK {
		return lastErr("gm_g16_stage_prove", rc)
	}
	return nil
}

// ProveR1CS proves from the staged wires through the resident R1CS r1 (a, b, c
// are evaluated on the device; gm_g16_stage_prove_r1cs).
func (st *G16Stage) ProveR1CS(r1 *R1CS, r, s, ar, bs, krs unsafe.Pointer) error {
	if rc := C.gm_g16_stage_prove_r1cs(st.h, r1.h, r, s, ar, bs, krs); rc != C.GM_OK {
		return lastErr("gm_g16_stage_prove_r1cs", rc)
	}
	return nil
}

// Free releases the stage (its buffers stay with the key for the next proof).
func (st *G16Stage) Free() { C.gm_g16_stage_free(st.h) }

// ---------------------------------------------------------------------------
// KZG (PLONK)
// ---------------------------------------------------------------------------

// SRS is a KZG SRS (pk.Kzg.G1 or pk.KzgLagrange.G1) resident on device 0.
type SRS struct {
	curve C.int
	dev   unsafe.Pointer
	n     int
}

// UploadSRS keeps the n G1Affine points at pts on the GPU.
func UploadSRS(curve int, pts unsafe.Pointer, n int) (*SRS, error) {
	ctx, err := Ctx()
	if err != nil {
		return nil, err
	}
	s := &SRS{curve: C.int(curve), n: n}
	if rc := C.gm_points_upload(ctx, C.int(curve), 0, pts, C.size_t(n), &s.dev); rc != C.GM_OK {
		return nil, lastErr("gm_points_upload", rc)
	}
	return s, nil
}

// Commit writes sum_i coeffs[i] * srs[i] (kzg.Commit) as a G1Affine at digest.
func (s *SRS) Commit(coeffs unsafe.Pointer, n int, digest unsafe.Pointer) error {
	if rc := C.gm_kzg_commit(ctx0, s.curve, s.dev, C.size_t(s.n), coeffs, C.size_t(n), digest); rc != C.GM_OK {
		return lastErr("gm_kzg_commit", rc)
	}
	return nil
}

// NTT runs an in-place fft.Domain FFT / FFTInverse of n fr.Elements at data
// (host memory; copied to and from device 0).
func NTT(curve int, data unsafe.Pointer, n int, inverse, dit, coset bool) error {
	ctx, err := Ctx()
	if err != nil {
		return err
	}
	b := func(v bool) C.int {
		if v {
			return 1
		}
		return 0
	}
	var dev unsafe.Pointer
	if rc := C.gm_copy_to_device(ctx, data, C.size_t(32*n), &dev); rc != C.GM_OK {
		return lastErr("gm_copy_to_device", rc)
	}
	defer C.gm_free(ctx, dev)
	if rc := C.gm_ntt(ctx, C.int(curve), dev, C.size_t(n), b(inverse), b(dit), b(coset)); rc != C.GM_OK {
		return lastErr("gm_ntt", rc)
	}
	if rc := C.gm_memcpy_d2h(ctx, data, dev, C.size_t(32*n)); rc != C.GM_OK {
		return lastErr("gm_memcpy_d2h", rc)
	}
	return nil
}
