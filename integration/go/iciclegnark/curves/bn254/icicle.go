// Package bn254 is a drop-in replacement for
// github.com/ingonyama-zk/iciclegnark/curves/bn254 v0.1.0 (go.mod:15 of the
// reference; not vendored there), binding the iciclegnark-semantics entries of
// libgnark_mi355x so backend/groth16/bn254/icicle/icicle.go runs UNCHANGED,
// frees included:
//
//   - INttOnDevice returns a NEW buffer holding natural-order coefficients and
//     leaves its input bit-reversed (icicle.go:489 frees that new buffer at :492,
//     :502's result is h);
//   - NttOnDevice(out, in) writes natural-order evaluations into out (:490);
//   - ReverseScalars(h) (:510) then yields the bit-reversed h pk.G1.Z expects.
//
// tests/test_icicle_replay_gpu.py replays icicle.go:453-513 and :231-412 call
// for call through exactly these C entries and matches the oracle's h and proof.
//
// NOT COMPILED HERE: this image has no Go toolchain.
package bn254

/*
#cgo CFLAGS: -I${SRCDIR}/../../../../../include
#cgo LDFLAGS: -L${SRCDIR}/../../../../../gnark-icicle_amd -lgnark_mi355x -Wl,-rpath,${SRCDIR}/../../../../../gnark-icicle_amd
#include "gnark_mi355x.h"
*/
import "C"

import (
	"fmt"
	"runtime"
	"sync"
	"unsafe"

	curve "github.com/consensys/gnark-crypto/ecc/bn254"
	"github.com/consensys/gnark-crypto/ecc/bn254/fr"
)

var (
	once sync.Once
	ctx  *C.gm_ctx
)

// One context (device 0, its own HIP stream).  C-ABI calls on a context are
// serialised inside the library, so icicle.go's goroutines may call
// concurrently.
func context() *C.gm_ctx {
	once.Do(func() {
		if rc := C.gm_init(0, &ctx); rc != C.GM_OK {
			panic("gnark_mi355x: " + C.GoString(C.gm_last_error()))
		}
	})
	return ctx
}

// iciclegnark has no error path for copies / NTTs / PolyOps (icicle.go never
// checks): a device failure there panics instead of corrupting a proof.
func must(rc C.int, what string) {
	if rc != C.GM_OK {
		panic(fmt.Sprintf("gnark_mi355x %s: %s", what, C.GoString(C.gm_last_error())))
	}
}

type OnDeviceData struct {
	P    unsafe.Pointer
	Size int
}

// CopyToDevice (icicle.go:44,47,65,245,269,352,478-480)
func CopyToDevice(s []fr.Element, bytes int, out chan unsafe.Pointer) {
	var p unsafe.Pointer
	must(C.gm_copy_to_device(context(), unsafe.Pointer(&s[0]), C.size_t(bytes), &p), "CopyToDevice")
	runtime.KeepAlive(s)
	out <- p
}

// CopyPointsToDevice (icicle.go:90,95,109,114): gnark G1Affine layout as is.
func CopyPointsToDevice(pts []curve.G1Affine, bytes int, out chan unsafe.Pointer) {
	var p unsafe.Pointer
	if len(pts) == 0 {
		must(C.gm_malloc(context(), 16, &p), "CopyPointsToDevice")
	} else {
		must(C.gm_copy_points_to_device(context(), C.GM_BN254, 0, unsafe.Pointer(&pts[0]), C.size_t(len(pts)), &p),
			"CopyPointsToDevice")
	}
	runtime.KeepAlive(pts)
	out <- p
}

// CopyG2PointsToDevice (icicle.go:125)
func CopyG2PointsToDevice(pts []curve.G2Affine, bytes int, out chan unsafe.Pointer) {
	var p unsafe.Pointer
	if len(pts) == 0 {
		must(C.gm_malloc(context(), 16, &p), "CopyG2PointsToDevice")
	} else {
		must(C.gm_copy_points_to_device(context(), C.GM_BN254, 1, unsafe.Pointer(&pts[0]), C.size_t(len(pts)), &p),
			"CopyG2PointsToDevice")
	}
	runtime.KeepAlive(pts)
	out <- p
}

// FreeDevicePointer (icicle.go:356,416-418,492,505-507)
func FreeDevicePointer(p unsafe.Pointer) {
	C.gm_free(context(), p)
}

// GenerateTwiddleFactors (icicle.go:68,73): builds the context's cached domain
// of size n; the returned pointer is a freeable handle standing for the table.
func GenerateTwiddleFactors(n int, inverse bool) (unsafe.Pointer, error) {
	var p unsafe.Pointer
	inv := C.int(0)
	if inverse {
		inv = 1
	}
	if rc := C.gm_icicle_generate_twiddles(context(), C.GM_BN254, C.size_t(n), inv, &p); rc != C.GM_OK {
		return nil, fmt.Errorf("GenerateTwiddleFactors: %s", C.GoString(C.gm_last_error()))
	}
	return p, nil
}

func cbool(b bool) C.int {
	if b {
		return 1
	}
	return 0
}

// INttOnDevice (icicle.go:489,502): natural-order evaluations at scalars_d ->
// a NEW device buffer of natural-order coefficients (coset: times g^-i); the
// domain tables come from the context (twiddles / coset-power pointers are the
// handles setupDevicePointers stored and are not read).
func INttOnDevice(scalars_d, twiddles_d, cosetPowers_d unsafe.Pointer, size, sizeBytes int, isCoset bool) unsafe.Pointer {
	var out unsafe.Pointer
	must(C.gm_icicle_intt_on_device(context(), C.GM_BN254, scalars_d, C.size_t(size), cbool(isCoset), &out),
		"INttOnDevice")
	return out
}

// NttOnDevice (icicle.go:490): natural-order coefficients at scalars_d ->
// natural-order evaluations (on the coset g*w^i) at scalars_out.
func NttOnDevice(scalars_out, scalars_d, twiddles_d, coset_powers_d unsafe.Pointer, size, twid_size, size_bytes int, isCoset bool) {
	must(C.gm_icicle_ntt_on_device(context(), C.GM_BN254, scalars_out, scalars_d, C.size_t(size), cbool(isCoset)),
		"NttOnDevice")
}

// PolyOps (icicle.go:500): a <- (a*b - c) * den, den the device vector
// pk.DenDevice (icicle.go:52-65).
func PolyOps(a_d, b_d, c_d, den_d unsafe.Pointer, size int) {
	must(C.gm_icicle_poly_ops(context(), C.GM_BN254, a_d, b_d, c_d, den_d, C.size_t(size)), "PolyOps")
}

// ReverseScalars (icicle.go:510)
func ReverseScalars(ptr unsafe.Pointer, n int) {
	must(C.gm_reverse_scalars(context(), C.GM_BN254, ptr, C.size_t(n)), "ReverseScalars")
}

// MsmOnDevice (icicle.go:302,315,332,355): scalars and gnark-layout points on
// the device; the result is gnark's G1Jac (same memory layout).
func MsmOnDevice(scalars_d, points_d unsafe.Pointer, count int, convert bool) (curve.G1Jac, unsafe.Pointer, error) {
	var out curve.G1Jac
	if rc := C.gm_msm(context(), C.GM_BN254, 0, scalars_d, points_d, C.size_t(count), unsafe.Pointer(&out), nil); rc != C.GM_OK {
		return out, nil, fmt.Errorf("MsmOnDevice: %s", C.GoString(C.gm_last_error()))
	}
	return out, nil, nil
}

// MsmG2OnDevice (icicle.go:382)
func MsmG2OnDevice(scalars_d, points_d unsafe.Pointer, count int, convert bool) (curve.G2Jac, unsafe.Pointer, error) {
	var out curve.G2Jac
	if rc := C.gm_msm(context(), C.GM_BN254, 1, scalars_d, points_d, C.size_t(count), unsafe.Pointer(&out), nil); rc != C.GM_OK {
		return out, nil, fmt.Errorf("MsmG2OnDevice: %s", C.GoString(C.gm_last_error()))
	}
	return out, nil, nil
}
