//go:build icicle

// GPU hooks for the BLS12-377 PLONK prover (BASELINE configs[4] "PLONK/KZG
// commit path"; the reference has no GPU path for PLONK, SURVEY.md §0.2).
//
// Seams in backend/plonk/bls12-377/prove.go, all behind the same
// backend.WithIcicleAcceleration() option (ProverConfig.Accelerator == "icicle"):
//
//  1. Every n-size MSM.  kzg.Commit(p, pk.KzgLagrange) at prove.go:312, 460 ->
//     commitLagrange; kzg.Commit(p, pk.Kzg) at :718 and the three quotient
//     commitments of commitToQuotient (:1154-1170) -> commitCanonical; the
//     opening quotients of kzg.Open (:611) and kzg.BatchOpenSinglePoint (:757)
//     -> open / batchOpen: the quotient polynomial is formed on the host exactly
//     as gnark-crypto's kzg does (Horner evaluation, synthetic division by
//     X - z), and only its commitment -- the MSM -- runs on the GPU (gm_kzg_commit
//     over the SRS kept resident, same digest bytes as kzg.Commit,
//     tests/test_msm_gpu.py::test_kzg_commit_and_prepared_msm).  The SRS is
//     selected explicitly by the caller, never by pointer identity.
//  2. Every n- and 4n-size FFT.  The domain0 ToCanonical / ToLagrange of
//     computeNumerator (:949, :967, :1016) and of computeLinearizedPolynomial
//     (:1301) -> toCanonical / toLagrange, and divideByZH's domain1 coset
//     FFTInverse (:1201) -> fftDomain1: gm.NTT with iop's decimation choice
//     (Regular -> DIF, BitReverse -> DIT: the layout flips, no bit reversal).
//
// Parity: the commits and transforms are replayed call for call against the
// oracle in tests/test_plonk_replay_gpu.py.  batchOpen's Fiat-Shamir challenge
// restates gnark-crypto's unexported kzg.deriveGamma (transcript "gamma":
// point, digests, claimed values, data); it cannot be compiled or run here (no
// Go toolchain), so every GPU batch opening is checked with gnark-crypto's own
// kzg.BatchVerifySinglePoint before it is used, and the CPU
// kzg.BatchOpenSinglePoint runs instead if the check fails.
//
// Wiring: prove.go.diff in this directory (a real patch against the
// reference's backend/plonk/bls12-377/prove.go; INTEGRATION.md §5).
// Without the icicle tag kzg_mi355x_stub.go keeps the patched file compiling
// (deviceFor returns nil and every call stays on gnark-crypto).
//
// NOT COMPILED HERE: this image has no Go toolchain.
package plonk

import (
	"errors"
	"hash"
	"os"
	"sync"
	"unsafe"

	curve "github.com/consensys/gnark-crypto/ecc/bls12-377"
	"github.com/consensys/gnark-crypto/ecc/bls12-377/fr"
	"github.com/consensys/gnark-crypto/ecc/bls12-377/fr/fft"
	"github.com/consensys/gnark-crypto/ecc/bls12-377/fr/iop"
	"github.com/consensys/gnark-crypto/ecc/bls12-377/kzg"
	fiatshamir "github.com/consensys/gnark-crypto/fiat-shamir"

	"github.com/consensys/gnark/backend/accel/mi355x/gm"
)

// kzgDevice keeps pk.Kzg.G1 and pk.KzgLagrange.G1 resident on the GPU (uploaded
// once per proving key, like setupDevicePointers does for Groth16).
type kzgDevice struct {
	once            sync.Once
	canonical, lagr *gm.SRS
	nCanon, nLagr   int
	vk              kzg.VerifyingKey
	err             error
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
		if len(pk.Kzg.G1) == 0 || len(pk.KzgLagrange.G1) == 0 || pk.Vk == nil {
			d.err = errors.New("gnark_mi355x: proving key without an SRS")
			return
		}
		if d.canonical, d.err = gm.UploadSRS(gm.BLS12_377, unsafe.Pointer(&pk.Kzg.G1[0]), len(pk.Kzg.G1)); d.err != nil {
			return
		}
		if d.lagr, d.err = gm.UploadSRS(gm.BLS12_377, unsafe.Pointer(&pk.KzgLagrange.G1[0]), len(pk.KzgLagrange.G1)); d.err != nil {
			return
		}
		d.nCanon, d.nLagr = len(pk.Kzg.G1), len(pk.KzgLagrange.G1)
		d.vk = pk.Vk.Kzg
	})
	return d.err
}

// commitWith replaces kzg.Commit(p, key) for the resident SRS srs of nSRS
// points: kzg.ErrInvalidPolynomialSize when p is longer, else the G1 digest
// sum_i p[i] * key.G1[i].
func commitWith(srs *gm.SRS, nSRS int, p []fr.Element) (kzg.Digest, error) {
	if len(p) > nSRS {
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

// commitLagrange: kzg.Commit(p, pk.KzgLagrange) (p in Lagrange form).
func (d *kzgDevice) commitLagrange(p []fr.Element) (kzg.Digest, error) {
	return commitWith(d.lagr, d.nLagr, p)
}

// commitCanonical: kzg.Commit(p, pk.Kzg) (p in canonical form).
func (d *kzgDevice) commitCanonical(p []fr.Element) (kzg.Digest, error) {
	return commitWith(d.canonical, d.nCanon, p)
}

// evalAt is p(z) by Horner (gnark-crypto kzg's eval).
func evalAt(p []fr.Element, z fr.Element) fr.Element {
	var r fr.Element
	for i := len(p) - 1; i >= 0; i-- {
		r.Mul(&r, &z).Add(&r, &p[i])
	}
	return r
}

// quotientByXminusZ returns (f(X) - fz) / (X - z), computed in place in f
// (synthetic division; the result is f[1:], of degree deg f - 1).  The
// quotient is unique, so its commitment is kzg.Open's H byte for byte.
func quotientByXminusZ(f []fr.Element, fz, z fr.Element) []fr.Element {
	f[0].Sub(&f[0], &fz)
	var t fr.Element
	for i := len(f) - 2; i >= 0; i-- {
		t.Mul(&f[i+1], &z)
		f[i].Add(&f[i], &t)
	}
	return f[1:]
}

// open replaces kzg.Open(p, z, pk.Kzg) (prove.go:611).
func (d *kzgDevice) open(p []fr.Element, z fr.Element) (kzg.OpeningProof, error) {
	if len(p) == 0 || len(p) > d.nCanon {
		return kzg.OpeningProof{}, kzg.ErrInvalidPolynomialSize
	}
	res := kzg.OpeningProof{ClaimedValue: evalAt(p, z)}
	q := make([]fr.Element, len(p))
	copy(q, p)
	h, err := d.commitCanonical(quotientByXminusZ(q, res.ClaimedValue, z))
	if err != nil {
		return kzg.OpeningProof{}, err
	}
	res.H.Set(&h)
	return res, nil
}

// deriveGamma restates gnark-crypto kzg's transcript for folding: challenge
// "gamma" bound to the point, the digests, the claimed values and the extra
// transcript data, in that order.
func deriveGamma(z fr.Element, digests []kzg.Digest, claimed []fr.Element, hf hash.Hash,
	data ...[]byte) (fr.Element, error) {
	fs := fiatshamir.NewTranscript(hf, "gamma")
	if err := fs.Bind("gamma", z.Marshal()); err != nil {
		return fr.Element{}, err
	}
	for i := range digests {
		if err := fs.Bind("gamma", digests[i].Marshal()); err != nil {
			return fr.Element{}, err
		}
	}
	for i := range claimed {
		if err := fs.Bind("gamma", claimed[i].Marshal()); err != nil {
			return fr.Element{}, err
		}
	}
	for i := range data {
		if err := fs.Bind("gamma", data[i]); err != nil {
			return fr.Element{}, err
		}
	}
	b, err := fs.ComputeChallenge("gamma")
	if err != nil {
		return fr.Element{}, err
	}
	var gamma fr.Element
	gamma.SetBytes(b)
	return gamma, nil
}

var errBatchCheck = errors.New("gnark_mi355x: GPU batch opening failed its verification")

// batchOpen replaces kzg.BatchOpenSinglePoint(polys, digests, z, hf, pk.Kzg,
// data...) (prove.go:757): claimed values f_i(z), gamma, the folded polynomial
// F = sum_i gamma^i f_i and its quotient (F - F(z)) / (X - z) on the host, the
// commitment on the GPU.  The result is checked with kzg.BatchVerifySinglePoint
// (gnark-crypto's own transcript); errBatchCheck tells the caller to use the
// CPU opening instead.
func (d *kzgDevice) batchOpen(polys [][]fr.Element, digests []kzg.Digest, z fr.Element, hf hash.Hash,
	data ...[]byte) (kzg.BatchOpeningProof, error) {
	if len(polys) != len(digests) || len(polys) == 0 {
		return kzg.BatchOpeningProof{}, kzg.ErrInvalidNbDigests
	}
	var res kzg.BatchOpeningProof
	res.ClaimedValues = make([]fr.Element, len(polys))
	largest := 0
	for i := range polys {
		if len(polys[i]) > d.nCanon {
			return kzg.BatchOpeningProof{}, kzg.ErrInvalidPolynomialSize
		}
		res.ClaimedValues[i] = evalAt(polys[i], z)
		if len(polys[i]) > largest {
			largest = len(polys[i])
		}
	}
	hf.Reset()
	gamma, err := deriveGamma(z, digests, res.ClaimedValues, hf, data...)
	if err != nil {
		return kzg.BatchOpeningProof{}, err
	}
	// F(z) = sum_i gamma^i f_i(z) and F = sum_i gamma^i f_i
	folded := res.ClaimedValues[len(polys)-1]
	for i := len(polys) - 2; i >= 0; i-- {
		folded.Mul(&folded, &gamma).Add(&folded, &res.ClaimedValues[i])
	}
	f := make([]fr.Element, largest)
	copy(f, polys[0])
	var gi, t fr.Element
	gi.SetOne()
	for i := 1; i < len(polys); i++ {
		gi.Mul(&gi, &gamma)
		for j := range polys[i] {
			t.Mul(&polys[i][j], &gi)
			f[j].Add(&f[j], &t)
		}
	}
	if res.H, err = d.commitCanonical(quotientByXminusZ(f, folded, z)); err != nil {
		return kzg.BatchOpeningProof{}, err
	}
	hf.Reset()
	if err := kzg.BatchVerifySinglePoint(digests, &res, z, hf, d.vk, data...); err != nil {
		return kzg.BatchOpeningProof{}, errBatchCheck
	}
	hf.Reset()
	return res, nil
}

// plainForm: a Lagrange or Canonical (not coset) polynomial of |dom|
// coefficients -- the only inputs the GPU transforms take; anything else
// (already in the target basis, coset forms, other sizes) goes to iop.
func plainForm(p *iop.Polynomial, dom *fft.Domain, from iop.Basis) bool {
	return p != nil && p.Basis == from && len(p.Coefficients()) == int(dom.Cardinality) &&
		os.Getenv("GNARK_MI355X_PLONK_FFT") != "0"
}

// toCanonical runs p.ToCanonical(dom) for a Lagrange p on the GPU: FFTInverse
// DIF on a Regular layout, DIT on a BitReverse one, and the layout flips (iop's
// choice: no bit-reversal pass).  false: the caller runs iop's transform.
func (d *kzgDevice) toCanonical(p *iop.Polynomial, dom *fft.Domain) bool {
	if !plainForm(p, dom, iop.Lagrange) {
		return false
	}
	c := p.Coefficients()
	dit := p.Layout == iop.BitReverse
	if gm.NTT(gm.BLS12_377, unsafe.Pointer(&c[0]), len(c), true, dit, false) != nil {
		return false
	}
	p.Basis = iop.Canonical
	p.Layout = flip(p.Layout)
	return true
}

// toLagrange: p.ToLagrange(dom) for a Canonical p (FFT, DIF / DIT as above).
func (d *kzgDevice) toLagrange(p *iop.Polynomial, dom *fft.Domain) bool {
	if !plainForm(p, dom, iop.Canonical) {
		return false
	}
	c := p.Coefficients()
	dit := p.Layout == iop.BitReverse
	if gm.NTT(gm.BLS12_377, unsafe.Pointer(&c[0]), len(c), false, dit, false) != nil {
		return false
	}
	p.Basis = iop.Lagrange
	p.Layout = flip(p.Layout)
	return true
}

func flip(l iop.Layout) iop.Layout {
	if l == iop.Regular {
		return iop.BitReverse
	}
	return iop.Regular
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
