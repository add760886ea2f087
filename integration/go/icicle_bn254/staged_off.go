//go:build icicle && !mi355x_levelhook

// Without the solver patch (tag mi355x_levelhook) there is no level hook: Prove
// sends the wires and a, b, c after Solve (or the wires only, with a, b, c
// evaluated from the resident R1CS).
package icicle_bn254

import (
	"errors"
	"unsafe"

	"github.com/consensys/gnark-crypto/ecc/bn254/fr"
	csolver "github.com/consensys/gnark/constraint/solver"

	"github.com/consensys/gnark/backend/accel/mi355x/gm"
)

type stagedRun struct{}

func (pk *ProvingKey) beginStaged(int, int, *gm.R1CS) (*stagedRun, csolver.Option, error) {
	return nil, nil, nil
}

func (run *stagedRun) prove([]fr.Element, *fr.Element, *fr.Element, unsafe.Pointer, unsafe.Pointer, unsafe.Pointer) error {
	return errors.New("gnark_mi355x: staged inputs need -tags mi355x_levelhook")
}

func (run *stagedRun) free() {}
