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
//  2. The domain1 (4n / 8n) transforms of the quotient computation
//     (prove.go:248-262, divideByZH :539) can call gm.NTT (fft.Domain FFT /
//     FFTInverse semantics, all DIF/DIT x coset modes; tests/test_ntt_gpu.py).
//
// Wiring (a patch to prove.go, shown in INTEGRATION.md §5): instance gains a
// `gpu *kzgDevice` field set in newInstance when opt.Accelerator == "icicle";
// every `kzg.Commit(x, key...)` call becomes `s.commit(x, key)`.
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
// inverse selects FFTInverse, dit the DIT decimation, coset fft.OnCoset().
func fftDomain1(v []fr.Element, inverse, dit, coset bool) error {
	if len(v) == 0 {
		return nil
	}
	return gm.NTT(gm.BLS12_377, unsafe.Pointer(&v[0]), len(v), inverse, dit, coset)
}
