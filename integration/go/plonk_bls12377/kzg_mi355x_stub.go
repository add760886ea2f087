//go:build !icicle

// Without the icicle build tag the patched prover (prove.go.diff) keeps
// compiling: deviceFor returns nil, so the instance never calls the methods
// below and every commit, opening and FFT stays on gnark-crypto's CPU path.
package plonk

import (
	"errors"
	"hash"

	"github.com/consensys/gnark-crypto/ecc/bls12-377/fr"
	"github.com/consensys/gnark-crypto/ecc/bls12-377/fr/fft"
	"github.com/consensys/gnark-crypto/ecc/bls12-377/fr/iop"
	"github.com/consensys/gnark-crypto/ecc/bls12-377/kzg"
)

type kzgDevice struct{}

func deviceFor(*ProvingKey) *kzgDevice { return nil }

var (
	errNoGPU      = errors.New("icicle backend requested but program compiled without 'icicle' build tag")
	errBatchCheck = errors.New("gnark_mi355x: GPU batch opening failed its verification")
)

func (d *kzgDevice) commitLagrange([]fr.Element) (kzg.Digest, error)  { return kzg.Digest{}, errNoGPU }
func (d *kzgDevice) commitCanonical([]fr.Element) (kzg.Digest, error) { return kzg.Digest{}, errNoGPU }

func (d *kzgDevice) open([]fr.Element, fr.Element) (kzg.OpeningProof, error) {
	return kzg.OpeningProof{}, errNoGPU
}

func (d *kzgDevice) batchOpen([][]fr.Element, []kzg.Digest, fr.Element, hash.Hash, ...[]byte) (kzg.BatchOpeningProof, error) {
	return kzg.BatchOpeningProof{}, errNoGPU
}

func (d *kzgDevice) toCanonical(*iop.Polynomial, *fft.Domain) bool { return false }
func (d *kzgDevice) toLagrange(*iop.Polynomial, *fft.Domain) bool  { return false }

func (d *kzgDevice) fftDomain1([]fr.Element, bool, bool, bool) error { return errNoGPU }
