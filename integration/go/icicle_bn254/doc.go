// Package icicle_bn254 implements MI355X (libgnark_mi355x) acceleration for the
// BN254 Groth16 backend behind backend.WithIcicleAcceleration(); drop-in for
// backend/groth16/bn254/icicle (doc.go:1-2).
package icicle_bn254
