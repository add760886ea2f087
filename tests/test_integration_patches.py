"""CPU checks of the Go-side patches under integration/go/ (no Go toolchain and
no gnark checkout here): the unified diff is well formed (every hunk's line
counts match its body, so `patch -p1` will not reject it as malformed) and it
rewires exactly the seams INTEGRATION.md §5 names in
backend/plonk/bls12-377/prove.go."""
import os
import re

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
DIFF = os.path.join(ROOT, "integration", "go", "plonk_bls12377", "prove.go.diff")


def _hunks(text):
    lines = text.split("\n")
    i = 0
    out = []
    while i < len(lines):
        m = re.match(r"^@@ -(\d+),(\d+) \+(\d+),(\d+) @@", lines[i])
        if not m:
            i += 1
            continue
        a_start, a_len, b_start, b_len = map(int, m.groups())
        body = []
        i += 1
        while i < len(lines) and not lines[i].startswith("@@") and not lines[i].startswith("--- "):
            body.append(lines[i])
            i += 1
        while body and body[-1] == "":
            body.pop()
        out.append((a_start, a_len, b_start, b_len, body))
    return out


def test_plonk_diff_is_well_formed():
    text = open(DIFF).read()
    assert "--- a/backend/plonk/bls12-377/prove.go" in text and "+++ b/backend/plonk/bls12-377/prove.go" in text
    hunks = _hunks(text)
    assert len(hunks) >= 8
    shift = 0
    for a_start, a_len, b_start, b_len, body in hunks:
        old = sum(1 for l in body if l[:1] in (" ", "-"))
        new = sum(1 for l in body if l[:1] in (" ", "+"))
        assert (old, new) == (a_len, b_len), (a_start, old, new, a_len, b_len)
        assert all(l[:1] in (" ", "-", "+", "\\") for l in body)
        assert b_start == a_start + shift, (a_start, b_start, shift)
        shift += b_len - a_len


def test_plonk_diff_rewires_every_msm_and_fft():
    """Every n-size MSM (kzg.Commit :312, 460, 718, 1158-1168; kzg.Open :611;
    kzg.BatchOpenSinglePoint :757) and every domain0 / domain1 FFT (:949, 967,
    1016, 1201, 1301) of backend/plonk/bls12-377/prove.go goes through the
    instance's hook; the only gnark-crypto calls left are the CPU fallbacks
    inside the helpers."""
    text = open(DIFF).read()
    removed = [l[1:] for l in text.split("\n") if l.startswith("-") and not l.startswith("---")]
    added = [l[1:] for l in text.split("\n") if l.startswith("+") and not l.startswith("+++")]
    code = [l for l in added if not l.strip().startswith("//")]
    assert sum("kzg.Commit(" in l for l in removed) == 6
    assert sum("kzg.Open(" in l for l in removed) == 1
    assert sum("kzg.BatchOpenSinglePoint(" in l for l in removed) == 1
    assert sum("s.commitLagrange(" in l for l in code) == 2      # :312, :460
    assert sum("s.commitCanonical(" in l for l in code) == 1     # :718
    assert any("commitToQuotient(s.h1(), s.h2(), s.h3(), s.proof, s.commitCanonical)" in l for l in code)
    assert sum(re.search(r"proof\.H\[\d\], err = commit\(h\d\)", l) is not None for l in code) == 3
    assert any("s.open(s.blindedZ, zetaShifted)" in l for l in code)
    assert any("s.batchOpen(" in l for l in code)
    # the domain0 transforms: three ToCanonical and one ToLagrange
    assert sum(re.search(r"\.To(Canonical|Lagrange)\(s\.domain0", l) is not None for l in removed) == 4
    assert sum("s.toCanonical0(" in l for l in code if "func" not in l) == 3
    assert sum("s.toLagrange0(" in l for l in code if "func" not in l) == 1
    assert any("gpu.fftDomain1(a.Coefficients(), true, true, true)" in l for l in added)
    assert any("a.ToCanonical(domains[1]).ToRegular()" in l for l in removed)
    assert any('opts.Accelerator == "icicle"' in l for l in added)
    # CPU fallbacks: exactly one call of each gnark-crypto entry, inside the helpers
    assert sum("kzg.Commit(" in l for l in code) == 2
    assert sum("kzg.Open(" in l for l in code) == 1
    assert sum("kzg.BatchOpenSinglePoint(" in l for l in code) == 1
    # the hook files the patch relies on exist for both build-tag variants
    d = os.path.dirname(DIFF)
    src = open(os.path.join(d, "kzg_mi355x.go")).read()
    stub = open(os.path.join(d, "kzg_mi355x_stub.go")).read()
    for name in ("func deviceFor(", "func (d *kzgDevice) commitLagrange(", "func (d *kzgDevice) commitCanonical(",
                 "func (d *kzgDevice) open(", "func (d *kzgDevice) batchOpen(", "func (d *kzgDevice) toCanonical(",
                 "func (d *kzgDevice) toLagrange(", "func (d *kzgDevice) fftDomain1(", "errBatchCheck"):
        assert name in src and name in stub, name
    assert src.startswith("//go:build icicle") and stub.startswith("//go:build !icicle")
    # the SRS is chosen by the method, never by comparing key pointers
    assert "== d.lagrKey" not in src and "*kzg.ProvingKey" not in src
