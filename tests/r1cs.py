"""Test circuits in R1CS (CSR) form, with their solved witnesses.

Shapes follow gnark's r1cs builder (frontend/cs/r1cs/api.go:199-212 -- one R1C
per Mul of two non-constant variables; api_assertions.go:30-44 -- AssertIsEqual
emits `1 * i1 == i2`) and the solver's wire order (constraint/bn254/solver.go:
73-119: ONE wire, public, secret, internal):

  * cubic_circuit()      examples/cubic/cubic.go:23-36 (x^3 + x + 5 == y), X=3, Y=35
  * squaring_chain(k)    backend/groth16/groth16_test.go:120-156 (refCircuit): k squarings of X
                         and AssertIsEqual(X_k, Y) -> k+1 constraints.

Solve (constraint/bn254/solver.go:426-532) is outside the hot path; the helpers
here compute the same W, a, b, c vectors directly for these circuits.
"""
from __future__ import annotations

import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "oracle"))
import pyref  # noqa: E402  (test oracle)


class R1CS:
    def __init__(self, curve: str, nb_public: int, nb_wires: int, constraints):
        """constraints: list of (L, R, O), each a list of (wire, coeff:int)."""
        self.curve = curve
        self.c = pyref.CURVES[curve]
        self.nb_public = nb_public
        self.nb_wires = nb_wires
        self.cons = constraints
        self.nc = len(constraints)
        n = 1
        while n < self.nc:
            n <<= 1
        self.domain_size = n
        self.rowptr, self.wires, self.coeffs = [], [], []
        for m in range(3):
            rp = [0]
            ws, cs = [], []
            for con in constraints:
                for w, co in con[m]:
                    ws.append(w)
                    cs.append(pyref.encode_fr(self.c, co))
                rp.append(len(ws))
            self.rowptr.append(np.array(rp, dtype=np.uint32))
            self.wires.append(np.array(ws if ws else [0], dtype=np.uint32))
            self.coeffs.append(np.frombuffer(b"".join(cs) if cs else bytes(32), dtype=np.uint8).copy())
        usedA = set(w for con in constraints for w, _ in con[0])
        usedB = set(w for con in constraints for w, _ in con[1])
        # exact infinity test happens in setup; for these circuits a wire is
        # non-zero in A(t) iff it appears in some L (coefficients are non-zero)
        self.nbA = len(usedA)
        self.nbB = len(usedB)

    def solve_abc(self, W):
        r = self.c.r
        a, b, cc = [], [], []
        for L, R, O in self.cons:
            a.append(sum(W[w] * co for w, co in L) % r)
            b.append(sum(W[w] * co for w, co in R) % r)
            cc.append(sum(W[w] * co for w, co in O) % r)
        return a, b, cc

    def is_satisfied(self, W):
        a, b, cc = self.solve_abc(W)
        return all(x * y % self.c.r == z for x, y, z in zip(a, b, cc))


def cubic_circuit(curve: str = "bn254"):
    # wires: 0 ONE, 1 Y (public), 2 X (secret), 3 t1 = X*X, 4 t2 = t1*X
    cons = [
        ([(2, 1)], [(2, 1)], [(3, 1)]),
        ([(3, 1)], [(2, 1)], [(4, 1)]),
        ([(0, 1)], [(1, 1)], [(4, 1), (2, 1), (0, 5)]),
    ]
    r1 = R1CS(curve, nb_public=2, nb_wires=5, constraints=cons)
    X = 3
    W = [1, 35, X, X * X, X * X * X]
    return r1, W


def squaring_chain(k: int, curve: str = "bn254", x: int = 2):
    # wires: 0 ONE, 1 Y, 2 X, 3..3+k-1 internals w_1..w_k
    cons = []
    for j in range(k):
        wj = 2 + j
        cons.append(([(wj, 1)], [(wj, 1)], [(wj + 1, 1)]))
    cons.append(([(0, 1)], [(2 + k, 1)], [(1, 1)]))
    r1 = R1CS(curve, nb_public=2, nb_wires=3 + k, constraints=cons)
    r = pyref.CURVES[curve].r
    W = [1, 0, x % r]
    v = x % r
    for _ in range(k):
        v = v * v % r
        W.append(v)
    W[1] = v
    return r1, W


def encode_vec(curve: str, vals) -> bytes:
    c = pyref.CURVES[curve]
    return b"".join(pyref.encode_fr(c, v) for v in vals)


class R1CSArrays:
    """R1CS in the CSR form the oracle consumes (same attributes as R1CS),
    built directly from numpy arrays -- for circuits with ~2^20 constraints,
    where the per-constraint Python lists of R1CS are too slow."""

    def __init__(self, curve, nb_public, nb_wires, nc, rowptr, wires, coeffs, nbA, nbB):
        self.curve = curve
        self.c = pyref.CURVES[curve]
        self.nb_public, self.nb_wires, self.nc = nb_public, nb_wires, nc
        n = 1
        while n < nc:
            n <<= 1
        self.domain_size = n
        self.rowptr, self.wires, self.coeffs = rowptr, wires, coeffs
        self.nbA, self.nbB = nbA, nbB


def squaring_chain_fast(k: int, curve: str = "bn254", x: int = 2):
    """squaring_chain(k) (groth16_test.go:120-156 refCircuit) as R1CSArrays plus
    the encoded solution: returns (r1, W, a, b, c), the last four as gnark-layout
    Montgomery bytes (W: nb_wires Fr; a, b, c: nc Fr each = solution.A/B/C)."""
    c = pyref.CURVES[curve]
    nc = k + 1
    one = pyref.encode_fr(c, 1)
    j = np.arange(k, dtype=np.uint32)
    rp = np.arange(nc + 1, dtype=np.uint32)  # exactly one term per row in L, R and O
    wl = np.concatenate([2 + j, np.array([0], np.uint32)])
    wr = np.concatenate([2 + j, np.array([2 + k], np.uint32)])
    wo = np.concatenate([3 + j, np.array([1], np.uint32)])
    co = np.frombuffer(one * nc, np.uint8).copy()
    r1 = R1CSArrays(curve, 2, 3 + k, nc, [rp, rp.copy(), rp.copy()], [wl, wr, wo], [co, co.copy(), co.copy()],
                    nbA=k + 1, nbB=k + 1)
    R = (1 << 256) % c.r
    v = x % c.r
    vals = [1, 0, v]
    for _ in range(k):
        v = v * v % c.r
        vals.append(v)
    vals[1] = v
    W = b"".join((u * R % c.r).to_bytes(32, "little") for u in vals)
    Wa = np.frombuffer(W, np.uint8).reshape(-1, 32)
    a = np.concatenate([Wa[2:2 + k], Wa[0:1]]).tobytes()
    b = np.concatenate([Wa[2:2 + k], Wa[2 + k:3 + k]]).tobytes()
    cc = np.concatenate([Wa[3:3 + k], Wa[1:2]]).tobytes()
    return r1, W, a, b, cc


def commitment_chain(k: int, curve: str = "bn254", ncommit: int = 1, x: int = 3):
    """squaring_chain(k) plus `ncommit` BSB22 commitments, the shape frontend
    api.Commit compiles to (the Bsb22CommitmentComputePlaceholder hint whose
    output wire is the commitment, prove.go:82-109; commitment info as in
    constraint/commitment.go:9-14):

      wires: 0 ONE, 1 Y (public), 2 X (secret), 3..2+k chain, then per
             commitment i: cm_i (commitment wire), u_i (internal)
      commitment i commits to private chain wires {2+i, 5+i, 8+i, ...} (every
             third wire, disjoint across commitments) and to the public Y; for
             i > 0 also to cm_{i-1} (a commitment-committed wire)
      constraints: the chain, AssertIsEqual(w_k, Y), and u_i = cm_i * v with
             v = X (i = 0) or u_{i-1}.

    Returns (r1, info, solve): solve(hint) fills W, calling
    hint(i, hashed_values, committed_values) -> commitment value (the
    overridden hint; `hashed` = PublicAndCommitmentCommitted values)."""
    assert k >= 3 * ncommit + 6
    nb_public = 2
    base = 3 + k
    cm = [base + 2 * i for i in range(ncommit)]
    u = [base + 2 * i + 1 for i in range(ncommit)]
    cons = []
    for j in range(k):
        wj = 2 + j
        cons.append(([(wj, 1)], [(wj, 1)], [(wj + 1, 1)]))
    cons.append(([(0, 1)], [(2 + k, 1)], [(1, 1)]))
    info = []
    for i in range(ncommit):
        priv = list(range(2 + i, 3 + k, 3 * ncommit))[:12]
        pac = [1] + ([cm[i - 1]] if i > 0 else [])
        info.append({"public_and_commitment_committed": pac, "nb_public_committed": 1,
                     "private_committed": sorted(priv), "commitment_index": cm[i]})
        v = 2 if i == 0 else u[i - 1]
        cons.append(([(cm[i], 1)], [(v, 1)], [(u[i], 1)]))
    r1 = R1CS(curve, nb_public=nb_public, nb_wires=base + 2 * ncommit, constraints=cons)
    r = pyref.CURVES[curve].r

    def solve(hint):
        W = [1, 0, x % r] + [0] * (k + 2 * ncommit)
        v = x % r
        for j in range(k):
            v = v * v % r
            W[3 + j] = v
        W[1] = v
        for i, ci in enumerate(info):
            hashed = [W[w] for w in ci["public_and_commitment_committed"]]
            W[cm[i]] = hint(i, hashed, [W[w] for w in ci["private_committed"]]) % r
            prev = W[2] if i == 0 else W[u[i - 1]]
            W[u[i]] = W[cm[i]] * prev % r
        assert r1.is_satisfied(W)
        return W

    return r1, info, solve
