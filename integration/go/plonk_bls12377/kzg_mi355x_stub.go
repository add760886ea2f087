//go:build !icicle

// Without the icicle build tag the patched prover (prove.go.diff) keeps
// compiling: no device, every commit / FFT stays on gnark-crypto's CPU path.
package plonk

import (
	"errors"

	"github.com/consensys/gnark-crypto/ecc/bls12-377/fr"
	"github.com/consensys/gnark-crypto/ecc/bls12-377/kzg"
)

type kzgDevice struct{}

func deviceFor(*ProvingKey) *kzgDevice { return nil }

var errNoGPU = errors.New("icicle backend requested but program compiled without 'icicle' build tag")

func (d *kzgDevice) commit([]fr.Element, *kzg.ProvingKey) (kzg.Digest, error) {
	return kzg.Digest{}, errNoGPU
}

func (d *kzgDevice) fftDomain1([]fr.Element, bool, bool, bool) error { return errNoGPU }
