"""The reference's own compiled constraint system, proved end to end.

internal/regression_tests/issue1045/testdata/issue1045.r1cs is the only
prover-side fixture the reference holds: a BN254 R1CS compiled by gnark's own
frontend (issue_1045_test.go:45-58 Circuit -- two public inputs, two hints,
two AssertIsEqual) and written by `ccs.WriteTo` (:63-77).  It is copied
verbatim to tests/golden/issue1045.r1cs (the GPU box has no /root/reference).

CPU: the reader (tests/gnark_r1cs.py) decodes every section consistently, the
CoeffTable holds gnark's fixed coefficients 0, 1, 2, -1, -2 (constraint/
coeff.go ids) in exactly the Montgomery bytes our encoder produces (a
reference-held pin of the Fr encoding), the solver restatement solves it with
In1 = 123, In2 = 333 and identity hints (issue_1045_test.go:25-33, :87-97),
and the oracle prover's proof passes the exponent-form verification.

GPU: the same system uploaded through gm_r1cs_upload (coefficient ids and the
fixture's own CoeffTable bytes) and proved with gm_g16_prove_r1cs, and proved
with gm_g16_prove from the solver's a, b, c: both proofs equal the oracle's
byte for byte and pass g16_check."""
import os

import pytest

import gnark_r1cs
import pyref
import r1cs as R

HERE = os.path.dirname(os.path.abspath(__file__))
FIXTURE = os.path.join(HERE, "golden", "issue1045.r1cs")
HINTS = {
    # issue_1045_test.go:19-22 (explicitHintName / anonymousHintName); both copy their input
    "github.com/consensys/gnark/internal/regression_tests/issue1045.ExplicitHint": lambda v: [v[0]],
    "github.com/consensys/gnark/internal/regression_tests/issue1045.glob..func1": lambda v: [v[0]],
}
TOXIC = [0x0F1E2D3C4B5A69788796A5B4C3D2E1F00F1E2D3C4B5A69788796A5B4C3D2E1,
         0x1122334455667788990011223344556677889900112233445566778899AABB,
         0x2233445566778899AABBCCDDEEFF00112233445566778899AABBCCDDEEFF01,
         0x13579BDF02468ACE13579BDF02468ACE13579BDF02468ACE13579BDF02468A,
         0x0102030405060708090A0B0C0D0E0F101112131415161718191A1B1C1D1E1F]


def _load():
    return gnark_r1cs.load(FIXTURE, pyref.BN254.r)


def _as_r1cs(sys_):
    return R.R1CS("bn254", nb_public=sys_.nb_public, nb_wires=sys_.nb_wires,
                  constraints=sys_.terms_by_value())


def test_issue1045_decodes():
    s = _load()
    assert s.version == (0, 10, 0) and s.gnark_version == "0.10.0"
    assert s.public == ["1", "In1", "In2"] and s.secret == [] and s.nb_internal == 2
    assert s.nb_constraints == 2 and s.nb_wires == 5
    assert s.blueprints == ["BlueprintGenericHint", "BlueprintGenericR1C"]
    assert sorted(s.hint_names.values()) == sorted(HINTS)
    assert s.commitments == []  # no BSB22 commitment
    # levels: both hints first, then both AssertIsEqual R1Cs
    assert s.levels == [[0, 1], [2, 3]]
    assert [i[0] for i in s.instructions] == ["hint", "hint", "r1c", "r1c"]
    # AssertIsEqual(res, In) compiles to 1 * res == In (frontend/cs/r1cs/api_assertions.go:30-44)
    assert s.constraints == [([(1, 0)], [(1, 3)], [(1, 1)]), ([(1, 0)], [(1, 4)], [(1, 2)])]


def test_issue1045_coeff_table_pins_fr_encoding():
    """gnark's CoeffTable starts with the fixed ids 0, 1, 2, -1, -2 (constraint/
    bn254/coeff.go:87-110); the fixture's bytes are those values in gnark-
    crypto's Montgomery form, which our encoder must reproduce exactly."""
    s = _load()
    r = pyref.BN254.r
    assert s.coeffs == [0, 1, 2, r - 1, r - 2]
    assert s.coeff_mont == [pyref.encode_fr(pyref.BN254, v) for v in s.coeffs]


def test_issue1045_solve():
    s = _load()
    W, a, b, c = s.solve([123, 333], [], HINTS)
    assert W == [1, 123, 333, 123, 333]
    assert (a, b, c) == ([1, 1], [123, 333], [123, 333])
    assert _as_r1cs(s).is_satisfied(W)
    with pytest.raises(ValueError, match="not satisfied"):
        s.solve([123, 333], [], dict(HINTS, **{k: (lambda v: [v[0] + 1]) for k in list(HINTS)[:1]}))
    with pytest.raises(ValueError, match="missing hint"):
        s.solve([123, 333], [], {})
    with pytest.raises(ValueError, match="witness size"):
        s.solve([123], [], HINTS)


def test_issue1045_reader_refuses_damage():
    data = open(FIXTURE, "rb").read()
    with pytest.raises(gnark_r1cs.R1CSFormatError):
        gnark_r1cs.GnarkR1CS(data[:-1], pyref.BN254.r)
    bad = bytearray(data)
    bad[8] = 1  # gnark major version 1
    with pytest.raises(gnark_r1cs.R1CSFormatError, match="version"):
        gnark_r1cs.GnarkR1CS(bytes(bad), pyref.BN254.r)
    with pytest.raises(gnark_r1cs.R1CSFormatError, match="scalar field"):
        gnark_r1cs.GnarkR1CS(data, pyref.CURVES["bls12377"].r)


def _oracle_proof(oracle, s, rr, ss):
    c = pyref.BN254
    r1 = _as_r1cs(s)
    W, a, b, cc = s.solve([123, 333], [], HINTS)
    enc = lambda v: R.encode_vec("bn254", v)
    tox = enc([t % c.r for t in TOXIC])
    pk = oracle.g16_setup("bn254", r1, tox)
    rb, sb = enc([rr]), enc([ss])
    exp = oracle.g16_prove("bn254", pk, r1.nb_public, enc(W), enc(a), enc(b), enc(cc), rb, sb)
    return r1, pk, tox, W, (a, b, cc), rb, sb, exp


def test_issue1045_oracle_prove_verifies(oracle):
    s = _load()
    r1, pk, tox, W, abc, rb, sb, exp = _oracle_proof(oracle, s, 0x5151, 0x7373)
    enc = lambda v: R.encode_vec("bn254", v)
    assert oracle.g16_check("bn254", r1, tox, enc(W), rb, sb, *exp) == 7
    # a proof for another witness does not verify against this one
    W2 = list(W)
    W2[1] = 124
    assert oracle.g16_check("bn254", r1, tox, enc(W2), rb, sb, *exp) != 7


@pytest.mark.gpu
@pytest.mark.parametrize("precompute", [False, True])
def test_issue1045_gpu_prove_r1cs_and_host_inputs(gm_ctx, oracle, precompute):
    import gnark_mi355x as gm
    s = _load()
    r1, pk, tox, W, (a, b, cc), rb, sb, exp = _oracle_proof(oracle, s, 0x2468ACE, 0x13579BD)
    enc = lambda v: R.encode_vec("bn254", v)
    dpk = gm.ProvingKey(gm_ctx, "bn254", pk, r1.domain_size, r1.nb_wires, r1.nb_public, precompute=precompute)
    csr = s.csr()
    h = gm.R1CS(gm_ctx, "bn254", s.nb_constraints, s.nb_wires, [m[0] for m in csr], [m[1] for m in csr],
                [m[2] for m in csr], b"".join(s.coeff_mont))
    try:
        got_r1cs = dpk.prove_r1cs(h, enc(W), rb, sb)
        got_host = dpk.prove(enc(W), enc(a), enc(b), enc(cc), rb, sb)
    finally:
        h.free()
        dpk.free()
    assert got_r1cs == exp
    assert got_host == exp
    assert oracle.g16_check("bn254", r1, tox, enc(W), rb, sb, *got_r1cs) == 7
