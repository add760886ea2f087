//go:build icicle

// GPU hooks for the BLS12-377 PLONK prover (BASELINE configs[4] "PLONK/KZG
// commit path"; the reference has no GPU path for PLONK, SURVEY.md §0.2).
//
// Two seams in backend/plonk/bls12-377/prove.go, both behind the same
// backend.WithIcicleAcceleration() option (ProverConfig.Accelerator == "icicle"):
//
//  1. kzg.Commit(p, pk.KzgLagrange) / kzg.Commit(p, pk.Kzg) at prove.go:312,
//     460, 718 and the three quotient commitments at 1158-1168 become
//     commit(...) below: an MSM of the coefficients against the SRS kept
//     resident on the GPU (gm_kzg_commit; same digest bytes as kzg.Commit,
//     tests/test_msm_gpu.py::test_kzg_commit_and_prepared_msm).
//  2. The domain1 (4n / 8n) transform of the quotient (domains prove.go:258-263,
//     divideByZH :1178-1205) calls gm.NTT (fft.Domain FFTInverse(DIT, OnCoset)
//     semantics; every DIF/DIT x coset mode is tested in tests/test_ntt_gpu.py;
//     the commit / FFT sequence is replayed in tests/test_plonk_replay_gpu.py).
//
// Wiring: prove.go.diff in this directory (a real patch against the
// reference's backend/plonk/bls12-377/prove.go; INTEGRATION.md §5): instance
// gains `gpu *kzgDevice`, set by deviceFor(pk) in newInstance when
// opt.Accelerator == "icicle"; every kzg.Commit goes through instance.commit;
// divideByZH runs its domain1 FFTInverse through fftDomain1.  Without the
// icicle tag kzg_mi355x_stub.go keeps the patched file compiling (gpu == nil).
//
// NOT COMPILED HERE: this image has no Go toolchain.
package plonk

import (
	"sync"
	"unsafe"

	curve "github.com/consensys/gnark-crypto/ecc/bls12-377"
	"github.com/consensys/gnark-crypto/ecc/bls12-377/fr"
	"github.com/consensys/gnark-crypto/ecc/bls12-377/kzg"

	"github.com/consensys/gnark/backend/accel/mi355x/gm"
)

// kzgDevice keeps pk.Kzg.G1 and pk.KzgLagrange.G1 resident on the GPU (uploaded
// once per proving key, like setupDevicePointers does for Groth16).
type kzgDevice struct {
	once              sync.Once
	canonical, lagr   *gm.SRS
	canonKey, lagrKey *kzg.ProvingKey
	err               error
}

// one kzgDevice per proving key (the SRS is uploaded once per key)
var devices sync.Map // *ProvingKey -> *kzgDevice

// deviceFor returns pk's device state, uploading its SRS on first use; nil when
// no GPU is usable (the prover then stays on the CPU path).
func deviceFor(pk *ProvingKey) *kzgDevice {
	v, _ := devices.LoadOrStore(pk, &kzgDevice{})
	d := v.(*kzgDevice)
	if d.setup(pk) != nil {
		return nil
	}
	return d
}

func (d *kzgDevice) setup(pk *ProvingKey) error {
	d.once.Do(func() {
		if d.canonical, d.err = gm.UploadSRS(gm.BLS12_377, unsafe.Pointer(&pk.Kzg.G1[0]), len(pk.Kzg.G1)); d.err != nil {
			return
		}
		d.lagr, d.err = gm.UploadSRS(gm.BLS12_377, unsafe.Pointer(&pk.KzgLagrange.G1[0]), len(pk.KzgLagrange.G1))
		d.canonKey, d.lagrKey = &pk.Kzg, &pk.KzgLagrange
	})
	return d.err
}

// commit replaces kzg.Commit(p, key): kzg.ErrInvalidPolynomialSize when p is
// longer than the SRS (gm_kzg_commit returns GM_ERR_INVALID), else the G1
// digest sum_i p[i] * key.G1[i].
func (d *kzgDevice) commit(p []fr.Element, key *kzg.ProvingKey) (kzg.Digest, error) {
	srs := d.canonical
	if key == d.lagrKey {
		srs = d.lagr
	}
	if len(p) > len(key.G1) {
		return kzg.Digest{}, kzg.ErrInvalidPolynomialSize
	}
	var out curve.G1Affine
	if len(p) == 0 {
		return out, nil
	}
	if err := srs.Commit(unsafe.Pointer(&p[0]), len(p), unsafe.Pointer(&out)); err != nil {
		return kzg.Digest{}, err
	}
	return out, nil
}

// fftDomain1 runs the domain1 transform of prove.go's quotient on the GPU:
// inverse selects FFTInverse, dit the DIT decimation, coset fft.OnCoset()
// (divideByZH: FFTInverse(DIT, OnCoset), bit-reversed in, natural out).
func (d *kzgDevice) fftDomain1(v []fr.Element, inverse, dit, coset bool) error {
	if len(v) == 0 {
		return nil
	}
	return gm.NTT(gm.BLS12_377, unsafe.Pointer(&v[0]), len(v), inverse, dit, coset)
}
