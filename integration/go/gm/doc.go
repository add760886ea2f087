// Package gm is the cgo binding of libgnark_mi355x (gm.go, build tag icicle).
// Without the tag the package is empty: nothing is compiled with cgo and
// nothing links -lgnark_mi355x, so gnark's default `go test ./...` is unchanged.
package gm
