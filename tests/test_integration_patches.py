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


def test_plonk_diff_rewires_every_commit_and_the_domain1_fft():
    text = open(DIFF).read()
    removed = [l[1:] for l in text.split("\n") if l.startswith("-") and not l.startswith("---")]
    added = [l[1:] for l in text.split("\n") if l.startswith("+") and not l.startswith("+++")]
    # prove.go:312, 460, 718 and the three quotient shards 1158-1168
    assert sum("kzg.Commit(" in l for l in removed) == 6
    assert sum("s.commit(" in l for l in added) == 3
    assert sum(re.search(r"proof\.H\[\d\], err = commit\(", l) is not None for l in added) == 3
    # the only kzg.Commit left is the CPU fallback inside instance.commit
    code = [l for l in added if not l.strip().startswith("//")]
    assert sum("kzg.Commit(" in l for l in code) == 1
    assert any("gpu.fftDomain1(a.Coefficients(), true, true, true)" in l for l in added)
    assert any("a.ToCanonical(domains[1]).ToRegular()" in l for l in removed)
    assert any('opts.Accelerator == "icicle"' in l for l in added)
    # the hook files the patch relies on exist for both build-tag variants
    d = os.path.dirname(DIFF)
    src = open(os.path.join(d, "kzg_mi355x.go")).read()
    stub = open(os.path.join(d, "kzg_mi355x_stub.go")).read()
    for name in ("func deviceFor(", "func (d *kzgDevice) commit(", "func (d *kzgDevice) fftDomain1("):
        assert name in src and name in stub, name
    assert src.startswith("//go:build icicle") and stub.startswith("//go:build !icicle")
