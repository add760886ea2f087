//go:build icicle && mi355x_levelhook

// Staged variant of Prove (SURVEY.md §8f row 4): the solver's results reach the
// GPU level by level while the R1CS solver still runs (constraint/bn254/solver.go:
// 426-532), so nothing crosses PCIe after Solve:
//   - the wires: every level's solved wire ids (wIDs) and the witness inputs,
//     scattered from solver.values into the stage's wire vector;
//   - a, b, c: every level's finished constraints, unless the constraint system
//     is resident on the device (then a, b, c are evaluated there from the staged
//     wires: gm_g16_stage_prove_r1cs).
// Needs the solver patch integration/go/solver_levelhook.diff
// (csolver.WithLevelHook); build with -tags icicle,mi355x_levelhook.
//
// NOT COMPILED HERE: this image has no Go toolchain.  The C side is tested by
// tests/test_pk_io_gpu.py::test_staged_inputs_by_level and
// tests/test_r1cs_gpu.py::test_groth16_stage_prove_r1cs_wires_by_level.
package icicle_bn254

import (
	"unsafe"

	"github.com/consensys/gnark-crypto/ecc/bn254/fr"
	csolver "github.com/consensys/gnark/constraint/solver"

	"github.com/consensys/gnark/backend/accel/mi355x/gm"
)

// stagedFlushAt is how many solved ids a level hook gathers before it hands
// them to the device stage in one call.  The reference's benchmark circuit
// (backend/groth16/groth16_test.go:120-156, a chain of squarings) solves one
// wire and one constraint per level (constraint/bn254/solver.go:471-484), so
// at 2^24 a call per level would be 2^24 cgo calls inside Solve; gathered, a
// level costs two appends.
const stagedFlushAt = 1 << 16

// stagedRun is one proof's staging area plus the first error a level hook hit.
type stagedRun struct {
	st        *gm.G16Stage
	r1        *gm.R1CS // resident constraint system (a, b, c evaluated on the device), or nil
	nbInputs  int      // witness wires [0, nbInputs): ONE, public, secret
	inputsPut bool
	perr      error
	// ids solved by levels and not yet handed over; values / a, b, c are the
	// solver's vectors, whose entries are final once their level is done
	pendW, pendC []uint32
	values       unsafe.Pointer
	a, b, c      unsafe.Pointer
}

// flushWires hands the gathered wire ids to the stage.
func (run *stagedRun) flushWires() error {
	if len(run.pendW) == 0 {
		return nil
	}
	err := run.st.PutIndexed(gm.StageWires, run.values, run.pendW)
	run.pendW = run.pendW[:0]
	return err
}

// flushConstraints hands the gathered constraint ids' a, b, c to the stage.
func (run *stagedRun) flushConstraints() error {
	if len(run.pendC) == 0 {
		return nil
	}
	for _, v := range []struct {
		which int
		base  unsafe.Pointer
	}{{gm.StageA, run.a}, {gm.StageB, run.b}, {gm.StageC, run.c}} {
		if err := run.st.PutIndexed(v.which, v.base, run.pendC); err != nil {
			return err
		}
	}
	run.pendC = run.pendC[:0]
	return nil
}

// beginStaged opens a staging area for nbConstraints constraints and returns
// the solver option that forwards every finished level to it.  r1 != nil: the
// constraint system is resident, only the wires are staged.
func (pk *ProvingKey) beginStaged(nbConstraints, nbInputs int, r1 *gm.R1CS) (*stagedRun, csolver.Option, error) {
	st, err := pk.deviceInfo.key.Stage(nbConstraints)
	if err != nil {
		return nil, nil, err
	}
	run := &stagedRun{st: st, r1: r1, nbInputs: nbInputs,
		pendW: make([]uint32, 0, stagedFlushAt), pendC: make([]uint32, 0, stagedFlushAt)}
	hook := func(cIDs []uint32, a, b, c unsafe.Pointer, wIDs []uint32, values unsafe.Pointer) {
		if run.perr != nil {
			return
		}
		run.values, run.a, run.b, run.c = values, a, b, c
		if !run.inputsPut { // the witness wires are solved before the first level
			if err := st.PutRange(gm.StageWires, 0, run.nbInputs, values); err != nil {
				run.perr = err
				return
			}
			run.inputsPut = true
		}
		run.pendW = append(run.pendW, wIDs...)
		if len(run.pendW) >= stagedFlushAt {
			if err := run.flushWires(); err != nil {
				run.perr = err
				return
			}
		}
		if run.r1 != nil || len(cIDs) == 0 {
			return
		}
		run.pendC = append(run.pendC, cIDs...) // cIDs is the solver's scratch: copied
		if len(run.pendC) >= stagedFlushAt {
			if err := run.flushConstraints(); err != nil {
				run.perr = err
			}
		}
	}
	return run, csolver.WithLevelHook(hook), nil
}

// prove is Prove's device block with the staged inputs: the solver ran with
// beginStaged's option, so every wire (and a, b, c) is already on its way to
// the device.
func (run *stagedRun) prove(w []fr.Element, r, s *fr.Element, ar, bs, krs unsafe.Pointer) error {
	if run.perr != nil {
		return run.perr
	}
	// what the last levels gathered
	if err := run.flushWires(); err != nil {
		return err
	}
	if err := run.flushConstraints(); err != nil {
		return err
	}
	if !run.inputsPut { // a system without levels: the hook never ran
		if err := run.st.PutRange(gm.StageWires, 0, len(w), unsafe.Pointer(&w[0])); err != nil {
			return err
		}
	}
	if run.r1 != nil {
		return run.st.ProveR1CS(run.r1, unsafe.Pointer(r), unsafe.Pointer(s), ar, bs, krs)
	}
	return run.st.Prove(unsafe.Pointer(r), unsafe.Pointer(s), ar, bs, krs)
}

func (run *stagedRun) free() { run.st.Free() }
