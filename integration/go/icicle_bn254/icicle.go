//go:build icicle

// Package icicle_bn254 -- MI355X build of backend/groth16/bn254/icicle.
//
// Re-derived from the CURRENT CPU prover groth16_bn254.Prove
// (backend/groth16/bn254/prove.go:62-325), not from the stale icicle.go
// (SURVEY.md §0.3: icicle.go:160 reads a HintID field constraint.Groth16Commitment
// no longer has, :44,47 read fft.Domain internals).  Everything before the
// device block is prove.go's own flow -- the BSB22 commitment hint, Solve, the
// proof-of-knowledge fold (prove.go:82-139) -- and the whole device block
// (computeH, compaction, 4 G1 + 1 G2 MSMs, finishing adds; prove.go:140-313,
// icicle.go:204-412) is ONE call into libgnark_mi355x: gm_g16_prove (one GPU) or
// gm_g16_prove_multi (the key sharded over every GPU of the node).
//
// NOT COMPILED HERE: this image has no Go toolchain.  The device block is the
// tested C-ABI (tests/test_groth16_gpu.py, tests/test_configs_full.py).
package icicle_bn254

import (
	"fmt"
	"math"
	"math/big"
	"os"
	"unsafe"

	"github.com/consensys/gnark-crypto/ecc"
	curve "github.com/consensys/gnark-crypto/ecc/bn254"
	"github.com/consensys/gnark-crypto/ecc/bn254/fr"
	"github.com/consensys/gnark-crypto/ecc/bn254/fr/hash_to_field"
	"github.com/consensys/gnark/backend"
	groth16_bn254 "github.com/consensys/gnark/backend/groth16/bn254"
	"github.com/consensys/gnark/backend/witness"
	"github.com/consensys/gnark/constraint"
	cs "github.com/consensys/gnark/constraint/bn254"
	"github.com/consensys/gnark/constraint/solver"
	fcs "github.com/consensys/gnark/frontend/cs"
	"github.com/consensys/gnark/logger"

	"github.com/consensys/gnark/backend/accel/mi355x/gm"
)

const HasIcicle = true

// kWires lists, for every point of pk.G1.K, the wire whose value multiplies it:
// the private wires minus the private-committed and commitment wires, i.e. the
// survivors of prove.go:243-245's filterHeap, as absolute wire indices.
func kWires(r1cs *cs.R1CS, nbWires int) []uint32 {
	info := r1cs.CommitmentInfo.(constraint.Groth16Commitments)
	drop := map[int]bool{}
	for _, i := range info.GetPrivateCommitted() {
		drop[i] = true
	}
	for _, i := range info.CommitmentIndexes() {
		drop[i] = true
	}
	if len(drop) == 0 {
		return nil // gm default: K[i] <-> wire nbPublic + i
	}
	out := make([]uint32, 0, nbWires)
	for i := r1cs.GetNbPublicVariables(); i < nbWires; i++ {
		if !drop[i] {
			out = append(out, uint32(i))
		}
	}
	return out
}

// setupDevicePointers uploads the key once (icicle.go:31-130).  The point arrays
// are converted to the MSM layout on the device.  GNARK_MI355X_PRECOMPUTE=1 /
// auto also keeps fixed-base window copies (always / when they fit the device:
// ~12x the point memory, -7% prove time at 2^24, +4.3 s of upload, so they pay
// off after ~440 proofs of one key; gm.PrecomputeFlags).
func (pk *ProvingKey) setupDevicePointers(r1cs *cs.R1CS) error {
	if pk.deviceInfo != nil {
		return nil
	}
	nbWires := len(pk.InfinityA)
	k := &gm.G16HostKey{
		DomainSize: pk.Domain.Cardinality, NbWires: uint64(nbWires),
		NbPublic: uint64(r1cs.GetNbPublicVariables()),
		NbA:      uint64(len(pk.G1.A)), NbB: uint64(len(pk.G1.B)), NbK: uint64(len(pk.G1.K)),
		Alpha:    unsafe.Pointer(&pk.G1.Alpha), Beta: unsafe.Pointer(&pk.G1.Beta), Delta: unsafe.Pointer(&pk.G1.Delta),
		Beta2:    unsafe.Pointer(&pk.G2.Beta), Delta2: unsafe.Pointer(&pk.G2.Delta),
		InfA:     pk.InfinityA, InfB: pk.InfinityB,
		KWires:   kWires(r1cs, nbWires),
	}
	// &s[0] of an empty slice would panic before any length test: take the
	// address only when there is an element
	g1 := func(s []curve.G1Affine) unsafe.Pointer {
		if len(s) == 0 {
			return nil
		}
		return unsafe.Pointer(&s[0])
	}
	k.A, k.B, k.Z, k.K = g1(pk.G1.A), g1(pk.G1.B), g1(pk.G1.Z), g1(pk.G1.K)
	if len(pk.G2.B) > 0 {
		k.B2 = unsafe.Pointer(&pk.G2.B[0])
	}
	flags := gm.PrecomputeFlags() // default: no window copies (gm.PrecomputeFlags)
	key, err := gm.UploadG16Key(gm.BN254, k, flags)
	if err != nil {
		return err
	}
	pk.deviceInfo = &deviceInfo{key: key}
	// the constraint system too (one GPU): proofs then send the wires alone.
	// It is an optimisation: if it cannot be uploaded (device memory after a
	// large precomputed key, term counts beyond u32) the proofs send a, b, c.
	if gm.NbDevices() == 1 && os.Getenv("GNARK_MI355X_R1CS") != "0" {
		r1, err := uploadR1CS(r1cs)
		if err != nil {
			logger.Logger().Warn().Err(err).Msg("mi355x: R1CS not resident, a/b/c are sent per proof")
		} else {
			pk.deviceInfo.r1 = r1
		}
	}
	return nil
}

// uploadR1CS hands r1cs.GetR1Cs() (constraint.R1C: L, R, O linear expressions
// of constraint.Term{CID, VID}; VID = MaxUint32 for a constant term, as
// GM_R1CS_CONST) and the CoeffTable to gm_r1cs_upload.
func uploadR1CS(r1cs *cs.R1CS) (*gm.R1CS, error) {
	rows := r1cs.GetR1Cs()
	if len(rows) == 0 || len(r1cs.Coefficients) == 0 {
		return nil, fmt.Errorf("empty constraint system")
	}
	var rowptr, cid, vid [3][]uint32
	for m := 0; m < 3; m++ {
		rowptr[m] = make([]uint32, 1, len(rows)+1)
	}
	for i := range rows {
		for m, l := range [3]constraint.LinearExpression{rows[i].L, rows[i].R, rows[i].O} {
			for _, t := range l {
				cid[m] = append(cid[m], t.CID)
				vid[m] = append(vid[m], t.VID)
			}
			// the row pointers are u32 (gm_r1cs_upload)
			if uint64(len(cid[m])) > math.MaxUint32 {
				return nil, fmt.Errorf("matrix %d has more than 2^32-1 terms", m)
			}
			rowptr[m] = append(rowptr[m], uint32(len(cid[m])))
		}
	}
	internal, secret, public := r1cs.GetNbVariables() // constraint/core.go:214
	return gm.UploadR1CS(gm.BN254, len(rows), internal+secret+public, rowptr, cid, vid,
		unsafe.Pointer(&r1cs.Coefficients[0]), len(r1cs.Coefficients))
}

// bsb22Hint is the BSB22 commitment hint of prove.go:82-109: it commits to the
// private committed values with the Pedersen key, hashes the commitment with
// the public/commitment-committed inputs to the field and returns that as the
// commitment wire's value.
func bsb22Hint(pk *ProvingKey, info constraint.Groth16Commitments, proof *groth16_bn254.Proof,
	committed [][]fr.Element, opt *backend.ProverConfig) solver.Hint {
	return func(_ *big.Int, in []*big.Int, out []*big.Int) error {
		i := int(in[0].Int64())
		args := in[1:]
		nbHashed := len(info[i].PublicAndCommitmentCommitted)
		hashed, priv := args[:nbHashed], args[nbHashed:]
		committed[i] = make([]fr.Element, len(info[i].PrivateCommitted))
		for j := range priv {
			committed[i][j].SetBigInt(priv[j])
		}
		var err error
		if proof.Commitments[i], err = pk.CommitmentKeys[i].Commit(committed[i]); err != nil {
			return err
		}
		h := opt.HashToFieldFn
		h.Write(constraint.SerializeCommitment(proof.Commitments[i].Marshal(), hashed, (fr.Bits-1)/8+1))
		digest := h.Sum(nil)
		h.Reset()
		take := fr.Bytes
		if h.Size() < take {
			take = h.Size()
		}
		var v fr.Element
		v.SetBytes(digest[:take])
		v.BigInt(out[0])
		return nil
	}
}

// foldPok computes proof.CommitmentPok (prove.go:113-139): one proof of
// knowledge per commitment key, folded with a challenge hashed from the
// commitment wires' values.
func foldPok(pk *ProvingKey, info constraint.Groth16Commitments, w []fr.Element, committed [][]fr.Element,
	proof *groth16_bn254.Proof) error {
	poks := make([]curve.G1Affine, len(pk.CommitmentKeys))
	for i := range pk.CommitmentKeys {
		var err error
		if poks[i], err = pk.CommitmentKeys[i].ProveKnowledge(committed[i]); err != nil {
			return err
		}
	}
	ser := make([]byte, fr.Bytes*len(info))
	for i := range info {
		copy(ser[fr.Bytes*i:], w[info[i].CommitmentIndex].Marshal())
	}
	challenge, err := fr.Hash(ser, []byte("G16-BSB22"), 1)
	if err != nil {
		return err
	}
	_, err = proof.CommitmentPok.Fold(poks, challenge[0], ecc.MultiExpConfig{NbTasks: 1})
	return err
}

// Prove generates the proof of knowledge of a r1cs with full witness (secret +
// public part) on the MI355X GPU(s).  Same signature, options, errors and proof
// bytes as groth16_bn254.Prove (given the same crypto/rand stream for r, s).
func Prove(r1cs *cs.R1CS, pk *ProvingKey, fullWitness witness.Witness, opts ...backend.ProverOption) (*groth16_bn254.Proof, error) {
	opt, err := backend.NewProverConfig(opts...)
	if err != nil {
		return nil, fmt.Errorf("new prover config: %w", err)
	}
	if opt.HashToFieldFn == nil {
		opt.HashToFieldFn = hash_to_field.New([]byte(constraint.CommitmentDst))
	}
	if opt.Accelerator != "icicle" {
		return groth16_bn254.Prove(r1cs, &pk.ProvingKey, fullWitness, opts...)
	}
	log := logger.Logger().With().Str("curve", r1cs.CurveID().String()).Str("acceleration", "mi355x").
		Int("nbConstraints", r1cs.GetNbConstraints()).Int("gpus", gm.NbDevices()).Str("backend", "groth16").Logger()
	if err := pk.setupDevicePointers(r1cs); err != nil {
		return nil, fmt.Errorf("setup device pointers: %w", err)
	}

	info := r1cs.CommitmentInfo.(constraint.Groth16Commitments)
	proof := &groth16_bn254.Proof{Commitments: make([]curve.G1Affine, len(info))}
	committed := make([][]fr.Element, len(info))
	solverOpts := append(opt.SolverOpts[:len(opt.SolverOpts):len(opt.SolverOpts)],
		solver.OverrideHint(solver.GetHintID(fcs.Bsb22CommitmentComputePlaceholder),
			bsb22Hint(pk, info, proof, committed, &opt)))

	// -tags mi355x_levelhook: the wires (and a, b, c unless the R1CS is resident)
	// move to the GPU level by level during Solve (staged.go); otherwise
	// beginStaged returns nil (staged_off.go)
	var staged *stagedRun
	if gm.NbDevices() == 1 {
		nbInputs := r1cs.GetNbPublicVariables() + r1cs.GetNbSecretVariables()
		st, hookOpt, err := pk.beginStaged(r1cs.GetNbConstraints(), nbInputs, pk.deviceInfo.r1)
		if err != nil {
			return nil, err
		}
		if st != nil {
			defer st.free()
			staged = st
			solverOpts = append(solverOpts, hookOpt)
		}
	}

	sol, err := r1cs.Solve(fullWitness, solverOpts...)
	if err != nil {
		return nil, err
	}
	solution := sol.(*cs.R1CSSolution)
	w := []fr.Element(solution.W)

	if err := foldPok(pk, info, w, committed, proof); err != nil {
		return nil, err
	}

	// r, s sampled exactly as prove.go:183-188 (same crypto/rand stream ->
	// byte-identical proofs on the CPU and the GPU path)
	var r, s fr.Element
	if _, err := r.SetRandom(); err != nil {
		return nil, err
	}
	if _, err := s.SetRandom(); err != nil {
		return nil, err
	}

	if staged != nil { // the wires (and a, b, c) already on the device
		if err := staged.prove(w, &r, &s, unsafe.Pointer(&proof.Ar), unsafe.Pointer(&proof.Bs),
			unsafe.Pointer(&proof.Krs)); err != nil {
			return nil, err
		}
		log.Debug().Msg("prover done")
		return proof, nil
	}
	if pk.deviceInfo.r1 != nil { // a, b, c come from the resident R1CS
		if err := pk.deviceInfo.key.ProveR1CS(pk.deviceInfo.r1, unsafe.Pointer(&w[0]), unsafe.Pointer(&r),
			unsafe.Pointer(&s), unsafe.Pointer(&proof.Ar), unsafe.Pointer(&proof.Bs), unsafe.Pointer(&proof.Krs)); err != nil {
			return nil, err
		}
		log.Debug().Msg("prover done")
		return proof, nil
	}
	nbCons := len(solution.A)
	if err := pk.deviceInfo.key.Prove(unsafe.Pointer(&w[0]), unsafe.Pointer(&solution.A[0]),
		unsafe.Pointer(&solution.B[0]), unsafe.Pointer(&solution.C[0]), nbCons,
		unsafe.Pointer(&r), unsafe.Pointer(&s),
		unsafe.Pointer(&proof.Ar), unsafe.Pointer(&proof.Bs), unsafe.Pointer(&proof.Krs)); err != nil {
		return nil, err
	}
	log.Debug().Msg("prover done")
	return proof, nil
}
