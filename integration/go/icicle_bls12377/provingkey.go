package icicle_bls12377

// MI355X GPU hook for backend/groth16/bls12-377 (new: the reference has none,
// SURVEY.md §0.2), shaped like backend/groth16/bn254/icicle/provingkey.go:1-36:
// no build tag and no cgo.  The key embeds the CPU key (so its serialization
// is the CPU key's) and a pointer to deviceInfo, defined per build-tag variant
// in device.go (icicle) and noicicle.go (!icicle).  Setup / DummySetup forward
// to the CPU setup.
//
// NOT COMPILED HERE: this image has no Go toolchain (tests/test_go_cgo_rules.py
// checks the build-tag sets statically).

import (
	groth16_bls12377 "github.com/consensys/gnark/backend/groth16/bls12-377"
	cs "github.com/consensys/gnark/constraint/bls12-377"
)

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
