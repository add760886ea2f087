//go:build icicle && mi355x_levelhook

// Staged variant of Prove (SURVEY.md §8f row 4): a, b, c reach the GPU level
// by level while the R1CS solver still runs (constraint/bn254/solver.go:
// 426-532), so the prove after Solve starts from device-resident inputs
// (gm_g16_stage_*).  Needs the solver patch integration/go/solver_levelhook.diff
// (csolver.WithLevelHook); build with -tags icicle,mi355x_levelhook.  Prove
// takes this path when the constraint system is not resident on the device.
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

// stagedRun is one proof's staging area plus the first error a level hook hit.
type stagedRun struct {
	st   *gm.G16Stage
	perr error
}

// beginStaged opens a staging area for nbConstraints constraints and returns
// the solver option that forwards every finished level's a[cID], b[cID],
// c[cID] to it.
func (pk *ProvingKey) beginStaged(nbConstraints int) (*stagedRun, csolver.Option, error) {
	st, err := pk.deviceInfo.key.Stage(nbConstraints)
	if err != nil {
		return nil, nil, err
	}
	run := &stagedRun{st: st}
	hook := func(cIDs []uint32, a, b, c unsafe.Pointer) {
		if run.perr != nil || len(cIDs) == 0 {
			return
		}
		for _, v := range []struct {
			which int
			base  unsafe.Pointer
		}{{gm.StageA, a}, {gm.StageB, b}, {gm.StageC, c}} {
			if err := st.PutIndexed(v.which, v.base, cIDs); err != nil {
				run.perr = err
				return
			}
		}
	}
	return run, csolver.WithLevelHook(hook), nil
}

// prove is Prove's device block with the staged inputs: the solver ran with
// beginStaged's option; only the wires are copied afterwards.
func (run *stagedRun) prove(w []fr.Element, r, s *fr.Element, ar, bs, krs unsafe.Pointer) error {
	if run.perr != nil {
		return run.perr
	}
	if err := run.st.PutRange(gm.StageWires, 0, len(w), unsafe.Pointer(&w[0])); err != nil {
		return err
	}
	return run.st.Prove(unsafe.Pointer(r), unsafe.Pointer(s), ar, bs, krs)
}

func (run *stagedRun) free() { run.st.Free() }
