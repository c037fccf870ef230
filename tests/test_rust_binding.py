"""The Rust crate's raw bindings (integration/fleetflow-placement/src/ffi.rs) must mirror
include/fleetplace.h: every #[repr(C)] struct field for field (name, order, type), every
declared function with the same parameter types, and the constants.  cargo is not in this
image, so this is the layout check that a header change without a matching ffi.rs change
fails ("a field reorder in the header would not fail any test")."""
import os
import re

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HDR = os.path.join(ROOT, "include", "fleetplace.h")
FFI = os.path.join(ROOT, "integration", "fleetflow-placement", "src", "ffi.rs")

C2R = {"uint32_t": "u32", "uint8_t": "u8", "uint64_t": "u64", "int64_t": "i64", "int": "c_int", "double": "f64", "void": "c_void",
       "char": "c_char", "fp_ctx": "fp_ctx", "fp_graph": "fp_graph", "fp_containers": "fp_containers",
       "fp_nodes": "fp_nodes", "fp_batch": "fp_batch"}


def _strip_c(src):
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return re.sub(r"//[^\n]*", "", src)


def c_type(base, const, stars):
    t = C2R[base]
    for i in range(stars):
        t = ("*const " if (const and i == 0) else "*mut ") + t
    return t


def header_structs():
    src = _strip_c(open(HDR).read())
    out = {}
    for body, name in re.findall(r"typedef struct\s*\{(.*?)\}\s*(\w+)\s*;", src, flags=re.S):
        fields = []
        for decl in body.split(";"):
            decl = decl.strip()
            if not decl:
                continue
            m = re.match(r"(const\s+)?(\w+)\s+(.*)", decl, flags=re.S)
            const, base, rest = bool(m.group(1)), m.group(2), m.group(3)
            for d in rest.split(","):
                d = d.strip()
                stars = d.count("*")
                fields.append((d.replace("*", "").strip(), c_type(base, const, stars)))
        out[name] = fields
    return out


def header_functions():
    src = _strip_c(open(HDR).read())
    out = {}
    for ret, name, args in re.findall(r"\n\s*((?:const\s+)?\w+\s*\**)\s*(fp_\w+)\s*\(([^)]*)\)\s*;", src):
        types = []
        for a in args.split(","):
            a = a.strip()
            if not a or a == "void":
                continue
            m = re.match(r"(const\s+)?(\w+)\s*(\**)\s*\w*$", a)
            types.append(c_type(m.group(2), bool(m.group(1)), len(m.group(3))))
        out[name] = types
    return out


def rust_structs():
    src = open(FFI).read()
    out = {}
    for name, body in re.findall(r"#\[repr\(C\)\]\s*pub struct (\w+)\s*\{(.*?)\}", src, flags=re.S):
        body = re.sub(r"//[^\n]*", "", body)
        out[name] = [(n, re.sub(r"\s+", " ", t).strip()) for n, t in re.findall(r"pub (\w+):\s*([^,]+),", body)]
    return out


def rust_functions():
    src = open(FFI).read()
    block = src[src.index("extern \"C\" {"):]
    out = {}
    for name, args in re.findall(r"pub fn (fp_\w+)\((.*?)\)", block, flags=re.S):
        out[name] = [re.sub(r"\s+", " ", t).strip() for t in re.findall(r"\w+:\s*([^,]+)", args)]
    return out


def test_every_header_struct_is_mirrored_field_for_field():
    hs, rs = header_structs(), rust_structs()
    assert set(hs) == {"fp_graph", "fp_containers", "fp_nodes", "fp_batch"}
    for name, fields in hs.items():
        assert rs.get(name) == fields, (name, fields, rs.get(name))


def test_every_header_function_is_bound_with_the_same_parameter_types():
    hf, rf = header_functions(), rust_functions()
    assert set(hf) == set(rf), (set(hf) ^ set(rf))
    for name, types in hf.items():
        got = [t.replace("f64", "f64") for t in rf[name]]
        assert got == types, (name, types, got)


def test_constants_match():
    src = _strip_c(open(HDR).read())
    rs = open(FFI).read()
    for name, val in re.findall(r"#define (FP_E\w+|FP_OK|FP_ABI_VERSION)\s+\(?(-?\d+)\)?", src):
        assert re.search(rf"pub const {name}: c_int = {val};", rs), name
    assert "pub const FP_NONE: u32 = 0xFFFF_FFFF;" in rs
    for name, val in re.findall(r"(FP_REASON_\w+) = (\d+)", src):
        assert re.search(rf"pub const {name}: u8 = {val};", rs), name
    for name, val in re.findall(r"(FP_K_(?!COUNT)\w+) = (\d+)", src):
        assert re.search(rf"pub const {name}: c_int = {val};", rs), name
    for name, val in re.findall(r"(FP_OPT_(?!COUNT)\w+) = (\d+)", src):
        assert re.search(rf"pub const {name}: c_int = {val};", rs), name
    for name, val in re.findall(r"(FP_GEOM_\w+) = (\d+)", src):
        assert re.search(rf"pub const {name}: usize = {val};", rs), name
    assert "pub const FP_OPT_AUTO: i64 = -1;" in rs


def _make_dry_run(*args):
    """The commands `make -B -n` would run in fleetflow_amd/csrc (nothing is built)."""
    import subprocess
    csrc = os.path.join(ROOT, "fleetflow_amd", "csrc")
    r = subprocess.run(["make", "-B", "-n", "-C", csrc, *args], capture_output=True, text=True, check=True)
    return [ln.strip() for ln in r.stdout.splitlines() if ln.strip() and not ln.startswith("make")]


def test_build_script_runs_the_makefile_recipe():
    """build.rs has no compiler command line of its own: it runs fleetflow_amd/csrc/Makefile with the
    objects and the library under cargo's OUT_DIR (a second copy of the recipe
    had drifted -- no -DFPP_SPLIT_BIG, no fp_pipe_big.hip under its own machine scheduler).  The
    Makefile's dry run with those two variables must be the in-tree recipe command for command
    (every translation unit with its own flags, the same link line) once the paths are mapped."""
    br = open(os.path.join(ROOT, "integration", "fleetflow-placement", "build.rs")).read()
    code = re.sub(r"//[^\n]*", "", br)
    assert 'Command::new("make")' in code
    assert '"BUILD={}"' in code and '"OUT={}"' in code and "arg(&src)" in code
    assert "offload-arch" not in code and ".hip" not in code  # no recipe of its own
    assert "rerun-if-changed={}\", src.display()" in code  # the whole source directory
    base = _make_dry_run()
    alt = _make_dry_run("BUILD=/cargo/out/obj", "OUT=/cargo/out/libfleetplace.so")
    mapped = [c.replace("/cargo/out/obj", "build").replace("/cargo/out/libfleetplace.so", "../libfleetplace.so")
              for c in alt]
    assert mapped == base
    compiles = [c for c in base if " -c " in c]
    mk = open(os.path.join(ROOT, "fleetflow_amd", "csrc", "Makefile")).read()
    srcs = re.search(r"SRCS := (.*)", mk).group(1).split()
    tus = _makefile_tus(mk)
    objs = [c.split(" -o ")[1].split()[0] for c in compiles]
    assert sorted(objs) == sorted([f"build/{s[:-4]}.o" for s in srcs] + [f"build/fp_pipe_tu_{t[0]}.o" for t in tus])
    by_obj = dict(zip(objs, compiles))
    assert "-DFPP_SPLIT" in by_obj["build/fp_pipe.o"]
    for name, g, blk, wv, pk, sched in tus:
        c = by_obj[f"build/fp_pipe_tu_{name}.o"]
        assert f"-DFPP_TU_NAME={name} -DFPP_TU_G={g} -DFPP_TU_BLK={blk} -DFPP_TU_WV={wv} -DFPP_TU_PK={pk}" in c
        assert (f"--amdgpu-sched-strategy={sched}" in c) == (sched != "default") and c.count("sched-strategy") <= 1
    link = [c for c in base if " -shared " in c and "../libfleetplace.so" in c]
    assert len(link) == 1 and all(o in link[0] for o in objs)


def _makefile_tus(mk):
    body = re.search(r"FFD_TUS := ((?:.*\\\n)*.*)", mk).group(1).replace("\\\n", " ")
    return [tuple(t.split(":")) for t in body.split()]


def test_kernel_translation_units_match_the_header_list():
    """The Makefile's FFD_TUS and fp_pipe_tus.h's FPP_TUS name the same kernels (name, G, BLK, WV,
    PK): fp_pipe.hip (FPP_SPLIT) declares a launcher for every header entry, and only the Makefile
    builds them."""
    mk = open(os.path.join(ROOT, "fleetflow_amd", "csrc", "Makefile")).read()
    hdr = open(os.path.join(ROOT, "fleetflow_amd", "csrc", "fp_pipe_tus.h")).read()
    listed = re.findall(r"X\((\w+), (\d+), (\d+), (\d+), (\d+)\)", hdr)
    assert listed and sorted(listed) == sorted(t[:5] for t in _makefile_tus(mk))


def _calls(src, prefix="ffi::"):
    """(name, number of top-level arguments) of every `ffi::fp_*(...)` call in src."""
    out = []
    for m in re.finditer(re.escape(prefix) + r"(fp_\w+)\(", src):
        i, depth, args, cur = m.end(), 1, 0, ""
        while depth:
            ch = src[i]
            if ch in "([{":
                depth += 1
            elif ch in ")]}":
                depth -= 1
            if depth == 1 and ch == ",":
                args += 1
                cur = ""
            elif depth >= 1:
                cur += ch
            i += 1
        nargs = 0 if not (cur.strip() or args) else args + 1
        out.append((m.group(1), nargs))
    return out


def test_every_ffi_call_in_lib_rs_is_declared_with_its_arity():
    """integration/fleetflow-placement/src/lib.rs calls only functions ffi.rs declares (i.e. the
    header declares), each with the declared number of arguments."""
    lib = open(os.path.join(ROOT, "integration", "fleetflow-placement", "src", "lib.rs")).read()
    rf, hf = rust_functions(), header_functions()
    calls = _calls(lib)
    assert {"fp_place_batch", "fp_dev_place_batch", "fp_dev_argmin_cost", "fp_place_ws_bytes"} <= {n for n, _ in calls}
    for name, nargs in calls:
        assert name in rf and name in hf, name
        assert nargs == len(hf[name]), (name, nargs, hf[name])
