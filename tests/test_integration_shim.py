"""INTEGRATION.md's R .Call shim (the reference-side binding of the C-ABI,
replacing NanoTel.R:2234-2258) type-checks against include/nanotel.h.  R is not
installed here, so the shim is compiled with gcc -fsyntax-only against
declarations of the R C API it uses (tests/r_api_decls); the library functions
it calls are the ones test_abi.py and test_rows_columns.py exercise."""
import os
import re
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.skipif(shutil.which("gcc") is None, reason="gcc not installed")
def test_r_shim_type_checks(tmp_path):
    text = open(os.path.join(ROOT, "INTEGRATION.md")).read()
    blocks = re.findall(r"```c\n(.*?)```", text, re.S)
    assert len(blocks) >= 2
    src = "\n".join(blocks)
    for fn in ("R_nt_create", "R_nt_analyze_chunk", "R_nt_filter_chunk", "nt_rows_columns",
               "nt_assign_serials", "nt_analyze_host"):
        assert fn in src, fn
    assert "omitted" not in src
    c = tmp_path / "nanotel_r.c"
    c.write_text(src)
    r = subprocess.run(["gcc", "-std=c11", "-fsyntax-only", "-Wall", "-Werror", "-Wno-unused-function",
                        "-I", os.path.join(ROOT, "include"), "-I", os.path.join(ROOT, "tests", "r_api_decls"),
                        str(c)], capture_output=True, text=True)
    assert r.returncode == 0, r.stderr
