package icicle_bls12377

// MI355X GPU hook for backend/groth16/bls12-377 (new: the reference has none, SURVEY.md §0.2)/provingkey.go: the key embeds
// the CPU key (so its serialization is the CPU key's, provingkey.go:25-28) and
// a handle to the device copy.  Setup / DummySetup forward to the CPU setup
// exactly as provingkey.go:30-36 does.
//
// NOT COMPILED HERE: this image has no Go toolchain.

import (
	"os"

	groth16_bls12377 "github.com/consensys/gnark/backend/groth16/bls12-377"
	cs "github.com/consensys/gnark/constraint/bls12-377"

	"github.com/consensys/gnark/backend/accel/mi355x/gm"
)

type deviceInfo struct {
	key *gm.G16Key
}

type ProvingKey struct {
	groth16_bls12377.ProvingKey
	*deviceInfo
}

func Setup(r1cs *cs.R1CS, pk *ProvingKey, vk *groth16_bls12377.VerifyingKey) error {
	return groth16_bls12377.Setup(r1cs, &pk.ProvingKey, vk)
}

func DummySetup(r1cs *cs.R1CS, pk *ProvingKey) error {
	return groth16_bls12377.DummySetup(r1cs, &pk.ProvingKey)
}

// FreeDevice releases the key's device copies (the reference keeps them for
// the process lifetime).
func (pk *ProvingKey) FreeDevice() {
	if pk.deviceInfo != nil {
		pk.deviceInfo.key.Free()
		pk.deviceInfo = nil
	}
}

func precomputeRequested() bool { return os.Getenv("GNARK_MI355X_PRECOMPUTE") == "1" }
