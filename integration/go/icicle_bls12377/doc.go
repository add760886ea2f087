// Package icicle_bls12377 implements MI355X (libgnark_mi355x) acceleration for
// the BLS12-377 Groth16 backend behind backend.WithIcicleAcceleration().
package icicle_bls12377
