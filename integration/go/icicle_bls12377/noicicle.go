//go:build !icicle

// Without the icicle build tag the package compiles with no cgo, mirroring
// backend/groth16/bn254/icicle/noicicle.go:1-18 for the second curve.
package icicle_bls12377

import (
	"errors"

	"github.com/consensys/gnark/backend"
	groth16_bls12377 "github.com/consensys/gnark/backend/groth16/bls12-377"
	"github.com/consensys/gnark/backend/witness"
	cs "github.com/consensys/gnark/constraint/bls12-377"
)

const HasIcicle = false

// deviceInfo holds nothing without a device.
type deviceInfo struct{}

func Prove(r1cs *cs.R1CS, pk *ProvingKey, fullWitness witness.Witness, opts ...backend.ProverOption) (*groth16_bls12377.Proof, error) {
	return nil, errors.New("icicle backend requested but program compiled without 'icicle' build tag")
}

func (pk *ProvingKey) FreeDevice() { pk.deviceInfo = nil }
