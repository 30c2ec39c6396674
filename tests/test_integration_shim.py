"""The R integration (r/): the .Call shim r/nanotel_r.c (the reference-side
binding of the C-ABI, replacing NanoTel.R:2234-2258), its R wrapper
r/nanotel.R and the patch r/NanoTel.R.patch.  R is not installed here, so the
shim is compiled with gcc -fsyntax-only against declarations of the R C API
it uses (tests/r_api_decls) and include/nanotel.h; the library functions it
calls are the ones test_abi.py and test_rows_columns.py exercise."""
import os
import re
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
R_DIR = os.path.join(ROOT, "r")
REF = "/root/reference/NanoTel.R"  # present in the build container only (read, never written)


@pytest.mark.skipif(shutil.which("gcc") is None, reason="gcc not installed")
def test_r_shim_type_checks():
    src = os.path.join(R_DIR, "nanotel_r.c")
    text = open(src).read()
    for fn in ("R_nt_create", "R_nt_analyze_chunk", "R_nt_filter_chunk", "nt_rows_columns",
               "nt_assign_serials", "nt_analyze_host", "nt_filter_host", "R_registerRoutines"):
        assert fn in text, fn
    r = subprocess.run(["gcc", "-std=c11", "-fsyntax-only", "-Wall", "-Wextra", "-Werror", "-Wno-unused-parameter",
                        "-Wno-cast-function-type",  # (DL_FUNC) casts: R's own registration idiom
                        "-I", os.path.join(ROOT, "include"), "-I", os.path.join(ROOT, "tests", "r_api_decls"),
                        src], capture_output=True, text=True)
    assert r.returncode == 0, r.stderr


def test_r_wrapper_calls_registered_entries():
    # every .Call of r/nanotel.R names a registered routine with that many arguments
    c = open(os.path.join(R_DIR, "nanotel_r.c")).read()
    reg = {m.group(1): int(m.group(2)) for m in re.finditer(r'\{"(R_nt_\w+)", \(DL_FUNC\)&\w+, (\d+)\}', c)}
    assert set(reg) == {"R_nt_create", "R_nt_destroy", "R_nt_analyze_chunk", "R_nt_filter_chunk"}
    for name, n in reg.items():  # the C definition takes that many SEXPs
        m = re.search(r"SEXP %s\(([^)]*)\)" % name, c)
        assert m and len(m.group(1).split(",")) == n, name
    rsrc = open(os.path.join(R_DIR, "nanotel.R")).read()
    calls = re.findall(r'\.Call\("(\w+)"((?:[^()]|\([^()]*(?:\([^()]*\))?[^()]*\))*)\)', rsrc)
    assert {nm for nm, _ in calls} == set(reg)
    for nm, args in calls:
        depth, count = 0, 0
        for ch in args:  # top-level commas of the argument list (after the name)
            depth += ch in "(["
            depth -= ch in ")]"
            count += ch == "," and depth == 0
        assert count == reg[nm], (nm, count)
    # the patch calls the wrapper's entry points and sources it
    patch = open(os.path.join(R_DIR, "NanoTel.R.patch")).read()
    for fn in ("nanotel_load()", "nanotel_create(", "nanotel_chunk(", "nanotel_filter("):
        assert fn in patch, fn
        assert fn.rstrip("()").rstrip("(") + " <- function" in rsrc, fn


@pytest.mark.skipif(not os.path.exists(REF) or shutil.which("patch") is None,
                    reason="the reference (build container only) or patch(1) absent")
def test_patch_applies_to_the_reference(tmp_path):
    # r/NanoTel.R.patch against NanoTel.R v1.1.9-beta: the per-chunk block
    # NanoTel.R:2234-2258 goes, nanotel_chunk() comes in, the rest stays
    dst = tmp_path / "NanoTel.R"
    shutil.copyfile(REF, dst)
    r = subprocess.run(["patch", str(dst), os.path.join(R_DIR, "NanoTel.R.patch")], capture_output=True, text=True)
    assert r.returncode == 0, r.stdout + r.stderr
    out = dst.read_text()
    assert "%<-%" not in out and "plan(multicore" not in out  # no forked workers left
    assert out.count("nanotel_chunk(") == 1 and "nanotel_create(" in out
    assert "write_csv" in out and "readDNAStringSet(files, nrec=nrec" in out  # the driver around it stays
