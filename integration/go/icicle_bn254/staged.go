//go:build icicle && mi355x_levelhook

// Staged variant of Prove (SURVEY.md §8f row 4): a, b, c reach the GPU level
// by level while the R1CS solver still runs (constraint/bn254/solver.go:
// 426-532), so the prove after Solve starts from device-resident inputs
// (gm_g16_stage_*).  Needs the 20-line solver patch of INTEGRATION.md §5
// (csolver.WithLevelHook); build with -tags icicle,mi355x_levelhook.
//
// NOT COMPILED HERE: this image has no Go toolchain.  The C side is tested by
// tests/test_pk_io_gpu.py::test_staged_inputs_by_level.
package icicle_bn254

import (
	"unsafe"

	"github.com/consensys/gnark-crypto/ecc/bn254/fr"
	csolver "github.com/consensys/gnark/constraint/solver"

	"github.com/consensys/gnark/backend/accel/mi355x/gm"
)

// stagedSolverOpts returns the solver option that forwards every finished
// level's a[cID], b[cID], c[cID] to st, and a function that reports the first
// error a put returned.
func stagedSolverOpts(st *gm.G16Stage) (csolver.Option, func() error) {
	var perr error
	hook := func(cIDs []uint32, a, b, c unsafe.Pointer) {
		if perr != nil || len(cIDs) == 0 {
			return
		}
		for _, v := range []struct {
			which int
			base  unsafe.Pointer
		}{{gm.StageA, a}, {gm.StageB, b}, {gm.StageC, c}} {
			if err := st.PutIndexed(v.which, v.base, cIDs); err != nil {
				perr = err
				return
			}
		}
	}
	return csolver.WithLevelHook(hook), func() error { return perr }
}

// proveStaged is Prove's device block with the staged inputs: the caller ran
// Solve with stagedSolverOpts(st); only the wires are copied afterwards.
func proveStaged(st *gm.G16Stage, w []fr.Element, r, s *fr.Element, ar, bs, krs unsafe.Pointer) error {
	if err := st.PutRange(gm.StageWires, 0, len(w), unsafe.Pointer(&w[0])); err != nil {
		return err
	}
	return st.Prove(unsafe.Pointer(r), unsafe.Pointer(s), ar, bs, krs)
}
