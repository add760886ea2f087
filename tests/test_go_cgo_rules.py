"""Static checks of the uncompiled Go seam (integration/go/) against the cgo
pointer-passing rules (no Go toolchain in this image, so these stand in for
`GODEBUG=cgocheck=1`).

Rule (cmd/cgo, Go >= 1.21): Go code may pass a Go pointer to C only if the Go
memory it points to contains no UNPINNED Go pointers.  A `C.<struct>{...}`
literal built in Go memory and passed by address (`&h`) therefore needs every
Go pointer stored in it pinned with a runtime.Pinner for the duration of the
call -- gm.go's G16HostKey.cHost does this for gm_g16_pk_host
(setupDevicePointers, backend/groth16/bn254/icicle/icicle.go:31-130).

A second, plain-Go trap is checked too: `f(len(s), &s[0])` evaluates `&s[0]`
before f can test the length, so an empty slice panics.
"""
import os
import re

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GO_DIR = os.path.join(ROOT, "integration", "go")


def go_files():
    for d, _, fs in os.walk(GO_DIR):
        for f in fs:
            if f.endswith(".go"):
                yield os.path.join(d, f)


def functions(src):
    """(header, body) of every top-level func, split on column-0 `func`."""
    parts = re.split(r"(?m)^func ", src)
    for p in parts[1:]:
        header = p.split("{", 1)[0]
        yield header, p


def struct_literals(body):
    """C.<name>{ ... } literals with their (brace-matched) text."""
    for m in re.finditer(r"C\.([A-Za-z_][A-Za-z0-9_]*)\{", body):
        i, depth = m.end(), 1
        while depth and i < len(body):
            depth += {"{": 1, "}": -1}.get(body[i], 0)
            i += 1
        yield m.group(1), m.start(), body[m.end():i - 1]


POINTERISH = re.compile(r"unsafe\.Pointer|&[A-Za-z_]|\bk\.(Alpha|Beta|Delta|A|B|Z|K|B2|Beta2|Delta2)\b")


def check_source(src, name="<src>"):
    """Violations of the rules above in one Go source text."""
    bad = []
    for header, body in functions(src):
        fname = header.split("(")[0].strip() or header[:40]
        has_pinner = "runtime.Pinner" in header or "runtime.Pinner" in body
        for sname, pos, lit in struct_literals(body):
            fields = [f.strip() for f in re.split(r",\s*\n|,(?![^()]*\))", lit) if ":" in f]
            for f in fields:
                key, val = f.split(":", 1)
                if val.strip().startswith("C.size_t(") or val.strip().startswith("C.int("):
                    continue
                if POINTERISH.search(val) and "pinned(" not in val:
                    bad.append(f"{name}:{fname}: C.{sname}.{key.strip()} holds an unpinned Go pointer: {val.strip()}")
            var = None
            mv = re.search(r"(\w+)\s*:?=\s*C\." + sname + r"\{", body[max(0, pos - 40):pos + len(sname) + 3])
            if mv:
                var = mv.group(1)
            if var:
                for am in re.finditer(r"\b" + var + r"\.(\w+)(?:\s*,\s*" + var + r"\.\w+)*\s*=\s*([^\n]+)", body):
                    rhs = am.group(2)
                    if POINTERISH.search(rhs) and "pinned(" not in rhs:
                        bad.append(f"{name}:{fname}: {var}.{am.group(1)} = {rhs.strip()} (unpinned Go pointer)")
                passed_by_addr = re.search(r"C\.\w+\(.*&" + var + r"\b", body) is not None
                if passed_by_addr and not has_pinner and POINTERISH.search(lit):
                    bad.append(f"{name}:{fname}: &{var} (C.{sname} with pointer fields) passed to C without a runtime.Pinner")
        # eager &s[0] in an argument list next to a length test
        for m in re.finditer(r"\w+\(len\((\w[\w.]*)\),\s*unsafe\.Pointer\(&\1\[0\]\)\)", body):
            bad.append(f"{name}:{fname}: {m.group(0)} evaluates &{m.group(1)}[0] before the length test")
    return bad


def test_go_seam_pins_go_pointers_in_c_structs():
    files = list(go_files())
    assert files, "integration/go is missing"
    bad = []
    for p in files:
        bad += check_source(open(p).read(), os.path.relpath(p, ROOT))
    assert not bad, "\n".join(bad)


def test_checker_catches_the_round2_pattern():
    # the shape gm.go had before the fix: Go pointers stored in a C struct
    # literal that is then passed by address, no Pinner
    src = '''
func UploadG16Key(curve int, k *G16HostKey, flags uint) (*G16Key, error) {
	infA := boolsToBytes(k.InfA)
	h := C.gm_g16_pk_host{
		nb_wires: C.size_t(k.NbWires),
		g1_alpha: k.Alpha,
		infA: (*C.uint8_t)(unsafe.Pointer(&infA[0])),
	}
	h.k_wires = (*C.uint32_t)(unsafe.Pointer(&k.KWires[0]))
	C.gm_g16_pk_upload_ex(ctx, C.int(curve), &h, C.uint(flags), &key.single)
	k.A = first(len(pk.G1.A), unsafe.Pointer(&pk.G1.A[0]))
}
'''
    bad = check_source(src)
    assert any("g1_alpha" in b for b in bad)
    assert any("infA" in b for b in bad)
    assert any("k_wires" in b for b in bad)
    assert any("without a runtime.Pinner" in b for b in bad)
    assert any("before the length test" in b for b in bad)


def test_gm_go_pins_every_host_key_pointer():
    src = open(os.path.join(GO_DIR, "gm", "gm.go")).read()
    m = re.search(r"func \(k \*G16HostKey\) cHost\(.*?\n}\n", src, re.S)
    assert m, "G16HostKey.cHost is missing"
    body = m.group(0)
    for field in ("g1_alpha", "g1_beta", "g1_delta", "g2_beta", "g2_delta", "g1_A", "g1_B", "g1_Z", "g1_K", "g2_B",
                  "infA", "infB", "k_wires"):
        assert field in body, field
    # both upload paths go through it and unpin after the call
    for fn in ("func UploadG16Key(", "func UploadG16KeyDump("):
        seg = src[src.index(fn):]
        seg = seg[:seg.index("\n}\n")]
        assert "var pin runtime.Pinner" in seg and "defer pin.Unpin()" in seg and "k.cHost(&pin" in seg, fn
