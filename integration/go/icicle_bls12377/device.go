//go:build icicle

// Device side of the BLS12-377 proving key (icicle build): the deviceInfo the
// untagged provingkey.go points at.
//
// NOT COMPILED HERE: this image has no Go toolchain.
package icicle_bls12377

import "github.com/consensys/gnark/backend/accel/mi355x/gm"

type deviceInfo struct {
	key *gm.G16Key
}

// FreeDevice releases the key's device copies (the reference keeps them for
// the process lifetime).
func (pk *ProvingKey) FreeDevice() {
	if pk.deviceInfo != nil {
		pk.deviceInfo.key.Free()
		pk.deviceInfo = nil
	}
}

