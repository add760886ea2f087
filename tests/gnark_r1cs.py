"""Reader for gnark's serialized R1CS (test infrastructure, not product code).

Parses the bytes `(*cs.R1CS).WriteTo` produces -- the reference's own fixture
internal/regression_tests/issue1045/testdata/issue1045.r1cs, written by
issue_1045_test.go:71-74 (`ccs.WriteTo(f)`), is copied to
tests/golden/issue1045.r1cs -- and restates the part of the solver the
Groth16 prover consumes, so that the HIP prover can be run on a constraint
system the reference compiled itself rather than on one this repo built.

Layout (all integers little-endian), following
  constraint/bn254/marshal.go:28-62   totalLen u64, gnark version major/minor/patch u64,
                                      System.ToBytes(), CoeffTable.toBytes()
  constraint/marshal.go:17-62,147-173 header {levelsLen, instructionsLen, calldataLen,
                                      bodyLen} u64, then the four sections
  constraint/marshal.go:234-250       levels: u64 count, then one compressed u32 array each
  constraint/marshal.go:192-232       instructions: compressed u32 BlueprintID,
                                      ConstraintOffset, WireOffset; compressed u64
                                      StartCallData
  constraint/marshal.go:175-190       calldata: u64 count, then uvarints
  constraint/marshal.go:128-145,335-363  body: CBOR (core deterministic) of
                                      constraint.System with tags 5309735+ for the
                                      blueprint types
  constraint/bn254/coeff.go:51-63     CoeffTable: u64 count, then 4 x u64 Montgomery limbs

The compressed arrays come from github.com/ronanh/intcomp (internal/backend/
ioutils/intcomp.go:12-32), a third-party module that is NOT vendored under
/root/reference (go.mod pins it; no module cache exists).  Only its
short-array form is restated, as observed in the fixture and cross-checked
against the calldata walk below: for arrays of fewer than 128 values the
words are [n, 3, packed..., 3] (u32; u64: [n | 2 << 32, packed..., 2]) and
the packed words hold the first-differences (from 0) one byte per value,
most significant byte first, padded with 0x80.  Longer arrays (bit-packed
blocks) are refused loudly rather than guessed.

The solver restated here (`solve`) follows constraint/bn254/solver.go:
newSolver :57-135 (wire order ONE, public, secret, internal; the witness
fills public-without-ONE then secret), run :426-532 (levels in order),
processInstruction :390-424 (R1C blueprint -> solveR1C, hint blueprint ->
solveWithHint), solveR1C :540-640 (a, b, c = <L,w>, <R,w>, <O,w>; at most one
unsolved wire, solved from a*b = c), the hint calldata of
constraint/blueprint_hint.go:10-36 and the R1C calldata of
constraint/blueprint_r1cs.go:20-59.
"""
from __future__ import annotations

import struct

# constraint/coeff.go fixed coefficient ids (CoeffIdZero .. CoeffIdMinusTwo)
COEFF_ZERO, COEFF_ONE, COEFF_TWO, COEFF_MINUS_ONE, COEFF_MINUS_TWO = 0, 1, 2, 3, 4
# constraint/marshal.go:340 first tag; order of addType calls :352-360
TAG_BASE = 5309735
TAG_NAMES = ["BlueprintGenericHint", "BlueprintGenericR1C", "BlueprintGenericSparseR1C",
             "BlueprintSparseR1CAdd", "BlueprintSparseR1CMul", "BlueprintSparseR1CBool",
             "BlueprintLookupHint", "Groth16Commitments", "PlonkCommitments"]


class R1CSFormatError(ValueError):
    pass


# --------------------------------------------------------------------------- CBOR (RFC 8949)
class Tagged:
    def __init__(self, tag, value):
        self.tag, self.value = tag, value

    def __repr__(self):
        return "Tagged(%d, %r)" % (self.tag, self.value)


def cbor_decode(buf: bytes, pos: int = 0):
    """Decodes one definite-length CBOR item; returns (value, next_pos)."""
    ib = buf[pos]
    major, info = ib >> 5, ib & 31
    pos += 1
    if info < 24:
        arg = info
    elif info in (24, 25, 26, 27):
        w = 1 << (info - 24)
        arg = int.from_bytes(buf[pos:pos + w], "big")
        pos += w
    else:
        raise R1CSFormatError("indefinite or reserved CBOR length at %d" % (pos - 1))
    if major == 0:
        return arg, pos
    if major == 1:
        return -1 - arg, pos
    if major == 2:
        return bytes(buf[pos:pos + arg]), pos + arg
    if major == 3:
        return buf[pos:pos + arg].decode("utf-8"), pos + arg
    if major == 4:
        out = []
        for _ in range(arg):
            v, pos = cbor_decode(buf, pos)
            out.append(v)
        return out, pos
    if major == 5:
        out = {}
        for _ in range(arg):
            k, pos = cbor_decode(buf, pos)
            v, pos = cbor_decode(buf, pos)
            out[k] = v
        return out, pos
    if major == 6:
        v, pos = cbor_decode(buf, pos)
        return Tagged(arg, v), pos
    # major 7
    simple = {20: False, 21: True, 22: None, 23: None}
    if info in simple:
        return simple[info], pos
    if info == 25:
        return struct.unpack(">e", arg.to_bytes(2, "big"))[0], pos
    if info == 26:
        return struct.unpack(">f", arg.to_bytes(4, "big"))[0], pos
    if info == 27:
        return struct.unpack(">d", arg.to_bytes(8, "big"))[0], pos
    raise R1CSFormatError("unsupported CBOR simple value %d" % info)


# --------------------------------------------------------------------------- intcomp short form
def _unpack_deltas(words, width, n):
    vals, prev = [], 0
    for w in words:
        for k in range(width // 8 - 1, -1, -1):
            if len(vals) == n:
                break
            byte = (w >> (8 * k)) & 0xFF
            if byte & 0x80:
                raise R1CSFormatError("intcomp: multi-byte delta (not in the restated short form)")
            prev += byte
            vals.append(prev)
    if len(vals) != n:
        raise R1CSFormatError("intcomp: %d values packed, %d expected" % (len(vals), n))
    return vals


def decompress_u32(words):
    """ioutils.ReadAndDecompressUints32's payload (intcomp.UncompressUint32), short form."""
    if not words:
        return []
    n = words[0]
    if n >= 128:
        raise R1CSFormatError("intcomp: bit-packed u32 blocks (n = %d) are not restated" % n)
    if len(words) != 3 + (n + 3) // 4 or words[1] != 3 or words[-1] != 3:
        raise R1CSFormatError("intcomp: unexpected u32 short-form framing %r" % (words,))
    return _unpack_deltas(words[2:-1], 32, n)


def decompress_u64(words):
    if not words:
        return []
    n, tag = words[0] & 0xFFFFFFFF, words[0] >> 32
    if n >= 128:
        raise R1CSFormatError("intcomp: bit-packed u64 blocks (n = %d) are not restated" % n)
    if len(words) != 2 + (n + 7) // 8 or tag != 2 or words[-1] != 2:
        raise R1CSFormatError("intcomp: unexpected u64 short-form framing %r" % (words,))
    return _unpack_deltas(words[1:-1], 64, n)


def _read_u32_array(buf, pos):
    """ioutils.ReadAndDecompressUints32 (intcomp.go:36-56): u64 word count, u32 words."""
    (length,) = struct.unpack_from("<Q", buf, pos)
    words = list(struct.unpack_from("<%dI" % length, buf, pos + 8))
    return decompress_u32(words), pos + 8 + 4 * length


def _read_u64_array(buf, pos):
    (length,) = struct.unpack_from("<Q", buf, pos)
    words = list(struct.unpack_from("<%dQ" % length, buf, pos + 8))
    return decompress_u64(words), pos + 8 + 8 * length


def _uvarint(buf, pos):
    """encoding/binary.Uvarint."""
    x, s = 0, 0
    while True:
        b = buf[pos]
        pos += 1
        x |= (b & 0x7F) << s
        if b < 0x80:
            return x, pos
        s += 7
        if s > 63:
            raise R1CSFormatError("uvarint overflow")


# --------------------------------------------------------------------------- the system
class GnarkR1CS:
    """A gnark BN254 R1CS as serialized by WriteTo."""

    def __init__(self, data: bytes, fr_modulus: int):
        self.r = fr_modulus
        total, major, minor, patch = struct.unpack_from("<4Q", data, 0)
        if major != 0 or minor < 10:  # constraint/bn254/marshal.go:82-84
            raise R1CSFormatError("unsupported gnark version %d.%d.%d" % (major, minor, patch))
        self.version = (major, minor, patch)
        if len(data) != 32 + total:
            raise R1CSFormatError("length %d, header says %d" % (len(data), 32 + total))
        sysb = data[32:]
        lv, ins, cd, body = struct.unpack_from("<4Q", sysb, 0)
        p = 32
        # levels (marshal.go:252-274)
        (nlev,) = struct.unpack_from("<Q", sysb, p)
        q = p + 8
        self.levels = []
        for _ in range(nlev):
            lvl, q = _read_u32_array(sysb, q)
            self.levels.append(lvl)
        if q != p + lv:
            raise R1CSFormatError("levels section length")
        p += lv
        # instructions (marshal.go:276-318)
        q = p
        self.blueprint_id, q = _read_u32_array(sysb, q)
        self.constraint_offset, q = _read_u32_array(sysb, q)
        self.wire_offset, q = _read_u32_array(sysb, q)
        self.start_calldata, q = _read_u64_array(sysb, q)
        if q != p + ins:
            raise R1CSFormatError("instructions section length")
        p += ins
        # calldata (marshal.go:320-333)
        (ncd,) = struct.unpack_from("<Q", sysb, p)
        q = p + 8
        self.calldata = []
        for _ in range(ncd):
            v, q = _uvarint(sysb, q)
            self.calldata.append(v)
        if q != p + cd:
            raise R1CSFormatError("calldata section length")
        p += cd
        # body (CBOR)
        self.body, q = cbor_decode(sysb, p)
        if q != p + body:
            raise R1CSFormatError("body length")
        p += body
        # CoeffTable (coeff.go:65-85)
        (nco,) = struct.unpack_from("<Q", sysb, p)
        p += 8
        self.coeff_mont = [bytes(sysb[p + 32 * i:p + 32 * i + 32]) for i in range(nco)]
        p += 32 * nco
        if p != len(sysb):
            raise R1CSFormatError("trailing bytes after the coefficient table")
        R_inv = pow(1 << 256, -1, self.r)
        self.coeffs = [int.from_bytes(c, "little") * R_inv % self.r for c in self.coeff_mont]

        b = self.body
        self.public = list(b["Public"])
        self.secret = list(b["Secret"] or [])
        self.nb_internal = b["NbInternalVariables"]
        self.nb_constraints = b["NbConstraints"]
        self.scalar_field = int(b["ScalarField"], 16)
        self.gnark_version = b["GnarkVersion"]
        self.blueprints = []
        for t in b["Blueprints"]:
            if not isinstance(t, Tagged) or not TAG_BASE <= t.tag < TAG_BASE + len(TAG_NAMES):
                raise R1CSFormatError("unknown blueprint %r" % (t,))
            self.blueprints.append(TAG_NAMES[t.tag - TAG_BASE])
        self.hint_names = {int(k): v for k, v in (b["MHintsDependencies"] or {}).items()}
        ci = b["CommitmentInfo"]
        self.commitments = ci.value if isinstance(ci, Tagged) else ci
        if self.scalar_field != self.r:
            raise R1CSFormatError("scalar field %x is not the expected curve's" % self.scalar_field)
        self._decode_instructions()

    @property
    def nb_public(self):
        return len(self.public)

    @property
    def nb_wires(self):
        return len(self.public) + len(self.secret) + self.nb_internal

    def _decode_instructions(self):
        """Walks the calldata per instruction (StartCallData; the first word of
        each instruction's calldata is its length for both blueprint kinds) and
        decodes R1Cs (blueprint_r1cs.go:36-59) and hints (blueprint_hint.go:10-36)."""
        n = len(self.blueprint_id)
        if not (len(self.constraint_offset) == len(self.wire_offset) == len(self.start_calldata) == n):
            raise R1CSFormatError("instruction arrays disagree")
        self.instructions = []
        walk = 0
        for i in range(n):
            s = self.start_calldata[i]
            if s != walk:
                raise R1CSFormatError("StartCallData[%d] = %d, calldata walk says %d" % (i, s, walk))
            size = self.calldata[s]
            cd = self.calldata[s:s + size]
            walk = s + size
            kind = self.blueprints[self.blueprint_id[i]]
            if kind == "BlueprintGenericR1C":
                nl, nr, no = cd[1], cd[2], cd[3]
                if size != 4 + 2 * (nl + nr + no):
                    raise R1CSFormatError("R1C calldata size")
                terms = [(cd[4 + 2 * k], cd[5 + 2 * k]) for k in range(nl + nr + no)]
                self.instructions.append(("r1c", self.constraint_offset[i],
                                          (terms[:nl], terms[nl:nl + nr], terms[nl + nr:])))
            elif kind == "BlueprintGenericHint":
                hid, nin = cd[1], cd[2]
                j, ins = 3, []
                for _ in range(nin):
                    ln = cd[j]
                    j += 1
                    ins.append([(cd[j + 2 * k], cd[j + 2 * k + 1]) for k in range(ln)])
                    j += 2 * ln
                start, end = cd[j], cd[j + 1]
                if j + 2 != size:
                    raise R1CSFormatError("hint calldata size")
                self.instructions.append(("hint", hid, (ins, start, end)))
            else:
                raise R1CSFormatError("blueprint %s is not restated" % kind)
        if walk != len(self.calldata):
            raise R1CSFormatError("calldata not fully consumed")
        seen = sorted(i for lvl in self.levels for i in lvl)
        if seen != list(range(n)):
            raise R1CSFormatError("levels do not cover every instruction exactly once")
        r1cs = [ins for ins in self.instructions if ins[0] == "r1c"]
        if sorted(c[1] for c in r1cs) != list(range(self.nb_constraints)):
            raise R1CSFormatError("constraint offsets are not 0..NbConstraints-1")
        self.constraints = [None] * self.nb_constraints
        for _, cid, lro in r1cs:
            self.constraints[cid] = lro

    # ---------------------------------------------------------------- evaluation
    def term_value(self, W, cid, vid):
        """computeTerm (solver.go:144-173) for a solved wire."""
        return self.coeffs[cid] * W[vid] % self.r

    def solve(self, public_witness, secret_witness, hints):
        """Returns (W, a, b, c) as integers; `hints` maps a hint NAME (as stored
        in MHintsDependencies) to f(inputs: list[int]) -> list[int] outputs."""
        r = self.r
        nw = self.nb_wires
        if len(public_witness) != len(self.public) - 1 or len(secret_witness) != len(self.secret):
            raise ValueError("invalid witness size")
        missing = [nm for nm in self.hint_names.values() if nm not in hints]
        if missing:
            raise ValueError("solver missing hint(s): %r" % missing)
        W = [None] * nw
        W[0] = 1
        for i, v in enumerate(list(public_witness) + list(secret_witness)):
            W[1 + i] = v % r
        a, b, c = [0] * self.nb_constraints, [0] * self.nb_constraints, [0] * self.nb_constraints
        for lvl in self.levels:
            for i in lvl:
                kind, key, payload = self.instructions[i]
                if kind == "hint":
                    ins, start, end = payload
                    vals = []
                    for le in ins:
                        acc = 0
                        for cid, vid in le:
                            if W[vid] is None:
                                raise ValueError("hint input wire %d unsolved" % vid)
                            acc += self.term_value(W, cid, vid)
                        vals.append(acc % r)
                    out = hints[self.hint_names[key]](vals)
                    if len(out) != end - start:
                        raise ValueError("hint output count")
                    for k, v in enumerate(out):
                        W[start + k] = v % r
                else:
                    self._solve_r1c(W, key, payload, a, b, c)
        if any(v is None for v in W):
            raise ValueError("not all wires were instantiated")
        return W, a, b, c

    def _solve_r1c(self, W, cid, lro, a, b, c):
        r = self.r
        acc = [0, 0, 0]
        unknown = None
        for m in range(3):
            for co, vid in lro[m]:
                if W[vid] is None:
                    if unknown is not None:
                        raise ValueError("found more than one wire to instantiate")
                    unknown = (m, co, vid)
                else:
                    acc[m] = (acc[m] + self.term_value(W, co, vid)) % r
        if unknown is not None:
            m, co, vid = unknown
            if m == 0:
                t = (acc[2] * pow(acc[1], -1, r) - acc[0]) % r
            elif m == 1:
                t = (acc[2] * pow(acc[0], -1, r) - acc[1]) % r
            else:
                t = (acc[0] * acc[1] - acc[2]) % r
            acc[m] = (acc[m] + t) % r
            W[vid] = t * pow(self.coeffs[co], -1, r) % r
        if acc[0] * acc[1] % r != acc[2]:
            raise ValueError("constraint #%d is not satisfied" % cid)
        a[cid], b[cid], c[cid] = acc

    def csr(self):
        """(rowptr, coeff_ids, wire_ids) per matrix L, R, O -- the form gm_r1cs_upload takes."""
        out = []
        for m in range(3):
            rp, ci, vi = [0], [], []
            for lro in self.constraints:
                for co, vid in lro[m]:
                    ci.append(co)
                    vi.append(vid)
                rp.append(len(ci))
            out.append((rp, ci, vi))
        return out

    def terms_by_value(self):
        """[(L, R, O)] with (wire, coefficient value) terms -- tests/r1cs.py's R1CS form."""
        return [tuple([(vid, self.coeffs[co]) for co, vid in lro[m]] for m in range(3))
                for lro in self.constraints]


def load(path: str, fr_modulus: int) -> GnarkR1CS:
    with open(path, "rb") as f:
        return GnarkR1CS(f.read(), fr_modulus)
