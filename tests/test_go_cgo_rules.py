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


# ---------------------------------------------------------------------------
# Build-tag completeness: gnark's default build (no tags,
# the reference CI `go test ./...`, .github/workflows/pr.yml:63-67) must compile
# the replacement packages WITHOUT cgo, exactly like the reference's
# provingkey.go:1-36 + noicicle.go:1-18; the icicle build must see one
# definition of every exported name.
# ---------------------------------------------------------------------------

TAG_SETS = [frozenset(), frozenset({"icicle"}), frozenset({"icicle", "mi355x_levelhook"})]
HOOK_PKGS = ("icicle_bn254", "icicle_bls12377")
GNARK_PKGS = HOOK_PKGS + ("gm", "plonk_bls12377")


def build_expr(src):
    """The //go:build expression of a Go file (None = untagged)."""
    for line in src.split("\n"):
        s = line.strip()
        if s.startswith("//go:build "):
            return s[len("//go:build "):].strip()
        if s.startswith("package "):
            return None
    return None


def eval_build(expr, tags):
    """Evaluate a //go:build expression (!, &&, ||, parentheses) for a tag set."""
    if expr is None:
        return True
    toks = re.findall(r"\(|\)|!|&&|\|\||[A-Za-z0-9_.]+", expr)
    pos = [0]

    def peek():
        return toks[pos[0]] if pos[0] < len(toks) else None

    def take():
        pos[0] += 1
        return toks[pos[0] - 1]

    def atom():
        t = take()
        if t == "!":
            return not atom()
        if t == "(":
            v = orx()
            assert take() == ")", expr
            return v
        return t in tags or t in ("linux", "amd64", "cgo", "gc")

    def andx():
        v = atom()
        while peek() == "&&":
            take()
            v = atom() and v
        return v

    def orx():
        v = andx()
        while peek() == "||":
            take()
            v = andx() or v
        return v

    v = orx()
    assert pos[0] == len(toks), expr
    return v


def strip_go(src):
    """Source without comments and string / rune literals."""
    src = re.sub(r"`[^`]*`", '""', src)
    src = re.sub(r'"(\\.|[^"\\\n])*"', '""', src)
    src = re.sub(r"'(\\.|[^'\\\n])+'", "0", src)
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return re.sub(r"//[^\n]*", "", src)


def imports(src):
    """Import paths of a Go file."""
    out = re.findall(r'(?m)^import\s+(?:\w+\s+)?"([^"]+)"', src)
    for block in re.findall(r"(?ms)^import \((.*?)^\)", src):
        out += re.findall(r'"([^"]+)"', block)
    return out


def top_decls(src):
    """Package-level declarations: names of funcs/types/consts/vars, and
    methods as Recv.name."""
    code = strip_go(src)
    out = []
    for m in re.finditer(r"(?m)^func\s+(?:\(\s*\w*\s*\*?(\w+)\s*\)\s*)?(\w+)", code):
        out.append(m.group(1) + "." + m.group(2) if m.group(1) else m.group(2))
    for kw in ("type", "const", "var"):
        for m in re.finditer(r"(?m)^" + kw + r"\s+(\w+)", code):
            out.append(m.group(1))
        for block in re.findall(r"(?ms)^" + kw + r" \((.*?)^\)", code):
            out += re.findall(r"(?m)^\t(\w+)", block)
    return out


def pkg_files(pkg):
    d = os.path.join(GO_DIR, pkg)
    return {f: open(os.path.join(d, f)).read() for f in sorted(os.listdir(d))
            if f.endswith(".go") and not f.endswith("_test.go")}


def included(pkg, tags):
    return {f: s for f, s in pkg_files(pkg).items() if eval_build(build_expr(s), tags)}


def test_build_expr_evaluator():
    assert eval_build(None, set())
    assert eval_build("!icicle", set()) and not eval_build("!icicle", {"icicle"})
    assert eval_build("icicle && !mi355x_levelhook", {"icicle"})
    assert not eval_build("icicle && !mi355x_levelhook", {"icicle", "mi355x_levelhook"})
    assert eval_build("(a || b) && !c", {"b"}) and not eval_build("(a || b) && !c", {"b", "c"})


def test_every_tag_set_defines_the_hook_api_once():
    for pkg in HOOK_PKGS:
        for tags in TAG_SETS:
            files = included(pkg, tags)
            seen = {}
            for f, s in files.items():
                for d in top_decls(s):
                    assert d not in seen, f"{pkg} {sorted(tags)}: {d} declared in {seen[d]} and {f}"
                    seen[d] = f
            for name in ("HasIcicle", "Prove", "ProvingKey", "Setup", "DummySetup", "deviceInfo",
                         "ProvingKey.FreeDevice"):
                assert name in seen, f"{pkg} {sorted(tags)}: {name} undefined"
            # one package clause for all included files
            pk = {re.search(r"(?m)^package (\w+)", s).group(1) for s in files.values()}
            assert pk == {pkg}, (pkg, pk)


def test_untagged_build_has_no_cgo_and_no_gm():
    for pkg in GNARK_PKGS:
        for f, s in included(pkg, frozenset()).items():
            imps = imports(s)
            assert "C" not in imps, f"{pkg}/{f}: untagged build imports \"C\""
            assert not any(i.endswith("/mi355x/gm") for i in imps), f"{pkg}/{f}: untagged build imports gm"
            assert "gm." not in strip_go(s), f"{pkg}/{f}: untagged build uses gm."


def test_names_used_are_declared_in_the_same_tag_set():
    """A package-level name (or method) declared under one tag set and used by
    a file of another set where it is not declared is a compile error."""
    for pkg in GNARK_PKGS:
        every = set()
        for s in pkg_files(pkg).values():
            every |= set(top_decls(s))
        plain = {d for d in every if "." not in d}
        methods = {d.split(".")[1] for d in every if "." in d}
        for tags in TAG_SETS:
            files = included(pkg, tags)
            have = set()
            for s in files.values():
                have |= set(top_decls(s))
            have_plain = {d for d in have if "." not in d}
            have_methods = {d.split(".")[1] for d in have if "." in d}
            for f, s in files.items():
                code = strip_go(s)
                for m in re.finditer(r"(?<![\w.])([A-Za-z_]\w*)\b", code):
                    name = m.group(1)
                    assert not (name in plain and name not in have_plain), \
                        f"{pkg}/{f} {sorted(tags)}: uses {name}, not declared in this tag set"
                for m in re.finditer(r"\.([a-z]\w*)\(", code):
                    name = m.group(1)
                    assert not (name in methods and name not in have_methods), \
                        f"{pkg}/{f} {sorted(tags)}: calls method {name}, not declared in this tag set"


def test_levelhook_diff_applies_to_the_reference_solver(tmp_path):
    """integration/go/solver_levelhook.diff (the csolver.WithLevelHook the
    staged prover needs) is a real patch: `patch --dry-run` applies it cleanly
    to the reference's constraint/solver/options.go and constraint/{bn254,
    bls12-377}/solver.go (copied to a temp dir; nothing under /root/reference
    is written)."""
    import shutil
    import subprocess
    import pytest
    ref = "/root/reference"
    diff = os.path.join(GO_DIR, "solver_levelhook.diff")
    text = open(diff).read()
    assert "func WithLevelHook(h LevelHook) Option" in text
    assert text.count("solver.levelDone(level)") == 4  # both branches of run(), both curves
    files = ["constraint/solver/options.go", "constraint/bn254/solver.go", "constraint/bls12-377/solver.go"]
    if not all(os.path.exists(os.path.join(ref, f)) for f in files) or shutil.which("patch") is None:
        pytest.skip("reference checkout or patch(1) not available")
    for f in files:
        (tmp_path / os.path.dirname(f)).mkdir(parents=True, exist_ok=True)
        shutil.copy(os.path.join(ref, f), tmp_path / f)
    r = subprocess.run(["patch", "-p1", "--dry-run", "-F0", "-i", diff], cwd=tmp_path, capture_output=True, text=True)
    assert r.returncode == 0 and "FAILED" not in r.stdout and "fuzz" not in r.stdout, r.stdout + r.stderr
    # the staged prover uses exactly the hook type the patch declares
    staged = open(os.path.join(GO_DIR, "icicle_bn254", "staged.go")).read()
    assert "csolver.WithLevelHook(hook)" in staged
    sig = "func(cIDs []uint32, a, b, c unsafe.Pointer, wIDs []uint32, values unsafe.Pointer)"
    assert sig in staged and "type LevelHook " + sig in text
    # every solved wire is logged where solver.set counts it, and each level's
    # log entries reach the hook (wires staged during Solve, not after it)
    assert text.count("s.wireLog[n-1-s.nbInputs] = uint32(id)") == 2
    assert text.count("wIDs := solver.wireLog[solver.logMark:end]") == 2
    # ... gathered (the squaring chain's one-wire levels cost two appends) and
    # handed over every stagedFlushAt ids and before the prove
    assert "run.pendW = append(run.pendW, wIDs...)" in staged
    assert "run.st.PutIndexed(gm.StageWires, run.values, run.pendW)" in staged
    assert "run.pendC = append(run.pendC, cIDs...)" in staged
    pv = staged[staged.index("func (run *stagedRun) prove("):]
    assert pv.index("run.flushWires()") < pv.index("ProveR1CS") and pv.index("run.flushConstraints()") < pv.index(
        "ProveR1CS")
    assert "PutRange(gm.StageWires, 0, len(w)" in staged  # only the no-level fallback
    # the diff is what tools/make_levelhook_patch.py generates from the reference
    import importlib.util
    spec = importlib.util.spec_from_file_location("mk", os.path.join(ROOT, "tools", "make_levelhook_patch.py"))
    mk = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mk)
    import difflib
    regen = []
    for rel, fn in (("constraint/bn254/solver.go", mk.patch_solver), ("constraint/bls12-377/solver.go",
                                                                     mk.patch_solver),
                    ("constraint/solver/options.go", mk.patch_options)):
        a = open(os.path.join(ref, rel)).read()
        regen += difflib.unified_diff(a.splitlines(True), fn(a).splitlines(True), "a/" + rel, "b/" + rel, n=3)
    assert "".join(regen) == text


def test_prove_diff_applies_to_the_reference_plonk_prover(tmp_path):
    import shutil
    import subprocess
    import pytest
    ref = "/root/reference/backend/plonk/bls12-377/prove.go"
    diff = os.path.join(GO_DIR, "plonk_bls12377", "prove.go.diff")
    if not os.path.exists(ref) or shutil.which("patch") is None:
        pytest.skip("reference checkout or patch(1) not available")
    dst = tmp_path / "backend/plonk/bls12-377"
    dst.mkdir(parents=True)
    shutil.copy(ref, dst / "prove.go")
    r = subprocess.run(["patch", "-p1", "--dry-run", "-F0", "-i", diff], cwd=tmp_path, capture_output=True, text=True)
    assert r.returncode == 0 and "FAILED" not in r.stdout and "fuzz" not in r.stdout, r.stdout + r.stderr


def test_install_into_a_reference_checkout(tmp_path):
    """integration/go/install.sh lays the seam into a copy of the reference
    gnark tree and applies all three patches; in the installed tree the
    untagged build of every touched package is cgo-free and the hook packages
    define their API once per tag set (the checks above, on the real layout)."""
    import shutil
    import subprocess
    import pytest
    ref = "/root/reference"
    if not os.path.exists(os.path.join(ref, "backend/groth16/groth16.go")) or shutil.which("patch") is None:
        pytest.skip("reference checkout or patch(1) not available")
    g = tmp_path / "gnark"
    shutil.copytree(ref, g, ignore=shutil.ignore_patterns(".git"))
    r = subprocess.run(["bash", os.path.join(GO_DIR, "install.sh"), str(g)], capture_output=True, text=True)
    assert r.returncode == 0, r.stdout + r.stderr
    src = (g / "backend/groth16/groth16.go").read_text()
    assert "icicle_bls12377.Prove(_r1cs, pk.(*icicle_bls12377.ProvingKey)" in src
    assert src.count("icicle_bls12377.HasIcicle") == 4  # Prove, Setup, DummySetup, NewProvingKey
    assert "WithLevelHook" in (g / "constraint/solver/options.go").read_text()
    for c in ("bn254", "bls12-377"):
        assert "solver.levelDone(level)" in (g / "constraint" / c / "solver.go").read_text()
    assert "s.commitLagrange(" in (g / "backend/plonk/bls12-377/prove.go").read_text()
    gm = (g / "backend/accel/mi355x/gm/gm.go").read_text()
    assert "#cgo CFLAGS: -I" + ROOT + "/include" in gm
    dirs = {"icicle_bn254": "backend/groth16/bn254/icicle", "icicle_bls12377": "backend/groth16/bls12-377/icicle"}
    for pkg, rel in dirs.items():
        d = g / rel
        names = sorted(f for f in os.listdir(d) if f.endswith(".go") and not f.endswith("_test.go"))
        assert names == sorted(pkg_files(pkg)), (pkg, names)  # the stale reference files are gone
        for tags in TAG_SETS:
            seen = set()
            for f in names:
                s = (d / f).read_text()
                if eval_build(build_expr(s), tags):
                    for dcl in top_decls(s):
                        assert dcl not in seen, (rel, sorted(tags), dcl)
                        seen.add(dcl)
            assert {"HasIcicle", "Prove", "ProvingKey", "Setup", "DummySetup", "deviceInfo"} <= seen
    # the reference's own package test keeps compiling against the new key type
    mt = (g / "backend/groth16/bn254/icicle/marshal_test.go").read_text()
    assert "icicle_bn254.Setup(tCcs, &iciPK, &iciVK)" in mt
    for rel in list(dirs.values()) + ["backend/accel/mi355x/gm", "backend/plonk/bls12-377"]:
        for f in os.listdir(g / rel):
            if f.endswith(".go"):
                s = (g / rel / f).read_text()
                if eval_build(build_expr(s), frozenset()):
                    assert "C" not in imports(s) and not any(i.endswith("/mi355x/gm") for i in imports(s)), (rel, f)


def test_every_import_is_used():
    """Go refuses unused imports; without a Go toolchain here, check that each
    imported package's name (alias or last path element) is referenced."""
    bad = []
    for p in go_files():
        src = open(p).read()
        code = strip_go(src)
        specs = re.findall(r'(?m)^import\s+(\w+\s+)?"([^"]+)"', src)
        for block in re.findall(r"(?ms)^import \((.*?)^\)", src):
            specs += re.findall(r'(?m)^\s*(\w+\s+|_\s+|\.\s+)?"([^"]+)"', block)
        for alias, path in specs:
            alias = alias.strip()
            if path == "C" or alias in ("_", "."):
                continue
            name = alias or path.rstrip("/").split("/")[-1]
            if name.startswith("v") and name[1:].isdigit():  # major-version suffix
                name = path.split("/")[-2]
            name = name.replace("-", "")
            if not re.search(r"\b" + re.escape(name) + r"\.", code):
                bad.append(f"{os.path.relpath(p, ROOT)}: import {path!r} ({name}) unused")
    assert not bad, "\n".join(bad)
