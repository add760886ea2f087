//go:build !icicle

// Without the icicle build tag the package compiles with no cgo, exactly as
// backend/groth16/bn254/icicle/noicicle.go:1-18: HasIcicle is false, so
// groth16.Prove (groth16.go:200-204) takes the CPU prover, and an explicit
// call to Prove returns the reference's error.
package icicle_bn254

import (
	"errors"
	"os"

	"github.com/consensys/gnark/backend"
	groth16_bn254 "github.com/consensys/gnark/backend/groth16/bn254"
	"github.com/consensys/gnark/backend/witness"
	cs "github.com/consensys/gnark/constraint/bn254"
)

const HasIcicle = false

// deviceInfo holds nothing without a device.
type deviceInfo struct{}

var errNoIcicle = errors.New("icicle backend requested but program compiled without 'icicle' build tag")

func Prove(r1cs *cs.R1CS, pk *ProvingKey, fullWitness witness.Witness, opts ...backend.ProverOption) (*groth16_bn254.Proof, error) {
	return nil, errNoIcicle
}

// The device-key helpers of device.go keep their signatures, so callers build
// in both tag sets.

func (pk *ProvingKey) FreeDevice() { pk.deviceInfo = nil }

func (pk *ProvingKey) ReadDumpToDevice(f *os.File, r1cs *cs.R1CS) error { return errNoIcicle }

func (pk *ProvingKey) SaveDeviceCache(f *os.File) error { return errNoIcicle }

func (pk *ProvingKey) LoadDeviceCache(f *os.File) error { return errNoIcicle }
