package icicle_bn254

// MI355X build of backend/groth16/bn254/icicle/provingkey.go: the key embeds
// the CPU key (so its serialization is the CPU key's, provingkey.go:25-28) and
// a handle to the device copy.  Setup / DummySetup forward to the CPU setup
// exactly as provingkey.go:30-36 does.
//
// NOT COMPILED HERE: this image has no Go toolchain.

import (
	"os"

	groth16_bn254 "github.com/consensys/gnark/backend/groth16/bn254"
	cs "github.com/consensys/gnark/constraint/bn254"

	"github.com/consensys/gnark/backend/accel/mi355x/gm"
)

type deviceInfo struct {
	key *gm.G16Key
}

type ProvingKey struct {
	groth16_bn254.ProvingKey
	*deviceInfo
}

func Setup(r1cs *cs.R1CS, pk *ProvingKey, vk *groth16_bn254.VerifyingKey) error {
	return groth16_bn254.Setup(r1cs, &pk.ProvingKey, vk)
}

func DummySetup(r1cs *cs.R1CS, pk *ProvingKey) error {
	return groth16_bn254.DummySetup(r1cs, &pk.ProvingKey)
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
