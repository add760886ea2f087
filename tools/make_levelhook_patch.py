#!/usr/bin/env python3
"""Regenerates integration/go/solver_levelhook.diff from the reference's solver
sources (read-only inputs; only the diff is written):

  constraint/solver/options.go       csolver.LevelHook / WithLevelHook
  constraint/bn254/solver.go         the hook call after every level, with the
  constraint/bls12-377/solver.go     level's R1C constraint ids (a, b, c final)
                                     and the ids of the wires solved in it

The wires of a level are logged by solver.set (solver.go:134-141), the one
place every solved wire goes through (hints :205-254, solveR1C :540-640,
SetValue :357-359): set already bumps nbSolved atomically, and that count
(minus the witness wires) is the wire's slot in an append-only log, so the
level's wires are the log entries added since the previous level.  Levels run
one after the other (run :426-532), so the hook sees every level complete.

  python tools/make_levelhook_patch.py [/root/reference]
"""
import difflib
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
OUT = os.path.join(ROOT, "integration", "go", "solver_levelhook.diff")


def sub(text, old, new, count=1):
    assert text.count(old) == count, (old[:60], text.count(old))
    return text.replace(old, new)


def patch_solver(src):
    s = sub(src, '\t"sync/atomic"\n', '\t"sync/atomic"\n\t"unsafe"\n')
    s = sub(s, '''	a, b, c fr.Vector // R1CS solver will compute the a,b,c matrices

	q *big.Int
}''', '''	a, b, c fr.Vector // R1CS solver will compute the a,b,c matrices

	levelHook csolver.LevelHook // called after each level (nil: no call)
	levelIDs  []uint32          // scratch: the R1C constraint ids of one level
	wireLog   []uint32          // level hook only: solved wire ids in solve order
	nbInputs  uint64            // wires solved before run (ONE + witness)
	logMark   uint64            // wireLog entries already handed to the hook

	q *big.Int
}''')
    s = sub(s, '''		nbTasks:         opt.NbTasks,
		q:               cs.Field(),''', '''		nbTasks:         opt.NbTasks,
		levelHook:       opt.LevelHook,
		q:               cs.Field(),''')
    s = sub(s, '''	s.nbSolved += uint64(len(witness) + witnessOffset)
''', '''	s.nbSolved += uint64(len(witness) + witnessOffset)
	if s.levelHook != nil {
		s.nbInputs = s.nbSolved
		s.wireLog = make([]uint32, nbWires-int(s.nbSolved))
	}
''')
    s = sub(s, '''	s.values[id] = value
	s.solved[id] = true
	atomic.AddUint64(&s.nbSolved, 1)
}''', '''	s.values[id] = value
	s.solved[id] = true
	n := atomic.AddUint64(&s.nbSolved, 1)
	if s.wireLog != nil {
		s.wireLog[n-1-s.nbInputs] = uint32(id)
	}
}''')
    s = sub(s, '''					return err
				}
			}
			continue
		}''', '''					return err
				}
			}
			solver.levelDone(level)
			continue
		}''')
    s = sub(s, '''		if len(chError) > 0 {
			return <-chError
		}
	}

	if int(solver.nbSolved) != len(solver.values) {''', '''		if len(chError) > 0 {
			return <-chError
		}
		solver.levelDone(level)
	}

	if int(solver.nbSolved) != len(solver.values) {''')
    s = sub(s, '''// solveR1C compute unsolved wires in the constraint, if any and set the solver accordingly''',
            '''// levelDone hands the level hook, if any, the constraint ids of the level's
// R1C instructions (one constraint each, at ConstraintOffset) and the wires the
// level solved (the wireLog entries since the previous level).
func (solver *solver) levelDone(level []uint32) {
	if solver.levelHook == nil || solver.Type != constraint.SystemR1CS || len(solver.a) == 0 {
		return
	}
	ids := solver.levelIDs[:0]
	for _, i := range level {
		pi := solver.Instructions[i]
		if _, ok := solver.Blueprints[pi.BlueprintID].(constraint.BlueprintR1C); ok {
			ids = append(ids, pi.ConstraintOffset)
		}
	}
	solver.levelIDs = ids
	end := atomic.LoadUint64(&solver.nbSolved) - solver.nbInputs
	wIDs := solver.wireLog[solver.logMark:end]
	solver.logMark = end
	if len(ids) > 0 || len(wIDs) > 0 {
		solver.levelHook(ids, unsafe.Pointer(&solver.a[0]), unsafe.Pointer(&solver.b[0]), unsafe.Pointer(&solver.c[0]),
			wIDs, unsafe.Pointer(&solver.values[0]))
	}
}

// solveR1C compute unsolved wires in the constraint, if any and set the solver accordingly''')
    return s


def patch_options(src):
    s = sub(src, '\t"runtime"\n', '\t"runtime"\n\t"unsafe"\n')
    s = sub(s, '''	NbTasks       int             // defaults to runtime.NumCPU()
}''', '''	NbTasks       int             // defaults to runtime.NumCPU()
	LevelHook     LevelHook       // defaults to nil (no call)
}

// LevelHook is called by the R1CS solver after every level of the solve:
// cIDs are the constraints whose a[cID], b[cID], c[cID] (fr.Element vectors
// at a, b, c) became final in that level, and wIDs the wires whose values
// (the fr.Element vector at values, indexed by wire id) were solved in it.
// The witness wires (ONE, public, secret: the first
// GetNbPublicVariables() + GetNbSecretVariables() of values) are solved before
// the first level.  The slices are only valid during the call; the solver does
// not run while the hook runs.
type LevelHook func(cIDs []uint32, a, b, c unsafe.Pointer, wIDs []uint32, values unsafe.Pointer)

// WithLevelHook is a solver option that registers a LevelHook, so a prover can
// move the solved wires and a, b, c to an accelerator while the next levels are
// solved.
func WithLevelHook(h LevelHook) Option {
	return func(opt *Config) error {
		opt.LevelHook = h
		return nil
	}
}''')
    return s


def main(ref):
    out = []
    for rel, fn in (("constraint/bn254/solver.go", patch_solver), ("constraint/bls12-377/solver.go", patch_solver),
                    ("constraint/solver/options.go", patch_options)):
        a = open(os.path.join(ref, rel)).read()
        b = fn(a)
        out += difflib.unified_diff(a.splitlines(True), b.splitlines(True), "a/" + rel, "b/" + rel, n=3)
    text = "".join(out)
    with open(OUT, "w") as f:
        f.write(text)
    print("wrote %s (%d lines)" % (OUT, text.count("\n")))


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "/root/reference")
