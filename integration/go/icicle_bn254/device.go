//go:build icicle

// Device side of the proving key (icicle build): the deviceInfo the untagged
// provingkey.go points at (reference provingkey.go:10-23 keeps raw device
// pointers there; here it is the libgnark_mi355x key handle), plus the key I/O
// helpers that stream a WriteDump file or a device-layout cache to the GPU.
//
// NOT COMPILED HERE: this image has no Go toolchain.
package icicle_bn254

import (
	"fmt"
	"io"
	"os"
	goUnsafe "unsafe"

	curve "github.com/consensys/gnark-crypto/ecc/bn254"
	"github.com/consensys/gnark-crypto/ecc/bn254/fr/pedersen"
	"github.com/consensys/gnark-crypto/utils/unsafe"
	cs "github.com/consensys/gnark/constraint/bn254"

	"github.com/consensys/gnark/backend/accel/mi355x/gm"
)

type deviceInfo struct {
	key *gm.G16Key
	r1  *gm.R1CS // resident constraint system (nil: a, b, c sent per proof)
}

// FreeDevice releases the key's device copies (the reference keeps them for
// the process lifetime).
func (pk *ProvingKey) FreeDevice() {
	if pk.deviceInfo != nil {
		pk.deviceInfo.key.Free()
		if pk.deviceInfo.r1 != nil {
			pk.deviceInfo.r1.Free()
		}
		pk.deviceInfo = nil
	}
}


// ReadDumpToDevice reads a key written by groth16_bn254.ProvingKey.WriteDump
// (backend/groth16/bn254/marshal.go:389-456) like ReadDump (:460-550) does,
// except that the five point slices are streamed from f straight into GPU
// memory (gm_g16_pk_upload_dump): the header is decoded here with the same
// gnark-crypto decoder, its byte count gives the offset of the first slice,
// and the commitment keys' slices after G2.B are read back into the Go key.
// pk.G1.A/B/Z/K and pk.G2.B stay empty; the device key replaces them.
func (pk *ProvingKey) ReadDumpToDevice(f *os.File, r1cs *cs.R1CS) error {
	cr := &countingReader{r: f}
	if err := unsafe.ReadMarker(cr); err != nil {
		return fmt.Errorf("read marker: %w", err)
	}
	if _, err := pk.Domain.ReadFrom(cr); err != nil {
		return fmt.Errorf("read domain: %w", err)
	}
	dec := curve.NewDecoder(cr, curve.NoSubgroupChecks())
	var nbWires uint64
	var nbCommitments uint32
	for i, v := range []interface{}{&pk.G1.Alpha, &pk.G1.Beta, &pk.G1.Delta, &pk.G2.Beta, &pk.G2.Delta,
		&nbWires, &pk.NbInfinityA, &pk.NbInfinityB} {
		if err := dec.Decode(v); err != nil {
			return fmt.Errorf("read field %d: %w", i, err)
		}
	}
	pk.InfinityA = make([]bool, nbWires)
	pk.InfinityB = make([]bool, nbWires)
	if err := dec.Decode(&pk.InfinityA); err != nil {
		return fmt.Errorf("read InfinityA: %w", err)
	}
	if err := dec.Decode(&pk.InfinityB); err != nil {
		return fmt.Errorf("read InfinityB: %w", err)
	}
	if err := dec.Decode(&nbCommitments); err != nil {
		return fmt.Errorf("read nbCommitments: %w", err)
	}
	nbPublic := r1cs.GetNbPublicVariables()
	kw := kWires(r1cs, int(nbWires))
	nbK := uint64(len(kw))
	if kw == nil {
		nbK = nbWires - uint64(nbPublic)
	}
	k := &gm.G16HostKey{
		DomainSize: pk.Domain.Cardinality, NbWires: nbWires, NbPublic: uint64(nbPublic),
		NbA:   nbWires - pk.NbInfinityA, NbB: nbWires - pk.NbInfinityB, NbK: nbK,
		Alpha: goUnsafe.Pointer(&pk.G1.Alpha), Beta: goUnsafe.Pointer(&pk.G1.Beta), Delta: goUnsafe.Pointer(&pk.G1.Delta),
		Beta2: goUnsafe.Pointer(&pk.G2.Beta), Delta2: goUnsafe.Pointer(&pk.G2.Delta),
		InfA:  pk.InfinityA, InfB: pk.InfinityB, KWires: kw,
	}
	flags := gm.PrecomputeFlags()
	key, end, err := gm.UploadG16KeyDump(gm.BN254, k, f, cr.n, flags)
	if err != nil {
		return err
	}
	pk.deviceInfo = &deviceInfo{key: key}
	if _, err := f.Seek(end, io.SeekStart); err != nil {
		return err
	}
	for i := 0; i < int(nbCommitments); i++ { // marshal.go:532-543
		cpkey := pedersen.ProvingKey{}
		if cpkey.Basis, _, err = unsafe.ReadSlice[[]curve.G1Affine](f); err != nil {
			return fmt.Errorf("read commitment basis %d: %w", i, err)
		}
		if cpkey.BasisExpSigma, _, err = unsafe.ReadSlice[[]curve.G1Affine](f); err != nil {
			return fmt.Errorf("read commitment basisExpSigma %d: %w", i, err)
		}
		pk.CommitmentKeys = append(pk.CommitmentKeys, cpkey)
	}
	return nil
}

// countingReader counts the header bytes the decoders consume (they read with
// io.ReadFull, no read-ahead), i.e. the offset of the first point slice.
type countingReader struct {
	r io.Reader
	n int64
}

func (c *countingReader) Read(p []byte) (int, error) {
	k, err := c.r.Read(p)
	c.n += int64(k)
	return k, err
}

// SaveDeviceCache / LoadDeviceCache persist the device copy of the key (with
// GNARK_MI355X_PRECOMPUTE window copies) in its device layout, so the
// conversion / precomputation runs once per key rather than once per process.
func (pk *ProvingKey) SaveDeviceCache(f *os.File) error {
	if pk.deviceInfo == nil {
		return fmt.Errorf("no device key")
	}
	return pk.deviceInfo.key.SaveCache(f)
}

func (pk *ProvingKey) LoadDeviceCache(f *os.File) error {
	key, err := gm.LoadG16KeyCache(gm.BN254, f)
	if err != nil {
		return err
	}
	pk.deviceInfo = &deviceInfo{key: key}
	return nil
}
