package icicle_bn254

// MI355X build of backend/groth16/bn254/icicle/provingkey.go:1-36.  Like the
// reference file it carries no build tag and no cgo: the key embeds the CPU key
// (so its serialization is the CPU key's, provingkey.go:25-28) and a pointer to
// deviceInfo, whose fields are defined per build-tag variant -- device.go
// (icicle: the libgnark_mi355x handles) and noicicle.go (!icicle: empty).  A
// plain `go test ./...` therefore neither compiles the cgo package gm nor
// links -lgnark_mi355x.  Setup / DummySetup forward to the CPU setup exactly
// as provingkey.go:30-36 does.
//
// NOT COMPILED HERE: this image has no Go toolchain (tests/test_go_cgo_rules.py
// checks the build-tag sets statically).

import (
	groth16_bn254 "github.com/consensys/gnark/backend/groth16/bn254"
	cs "github.com/consensys/gnark/constraint/bn254"
)

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
