#!/usr/bin/env python3
"""Fill the on-disk hiprtc cache (nanotel_amd/jitcache) with the code objects of
the GPU tests' pattern sets that wait for the specialised calling kernel
(NT_CALL_JIT=1), so a GPU run does not spend its time limit in hiprtc.  Runs on
the CPU (no device needed), one process per pattern set."""
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.join(HERE, "..")
sys.path.insert(0, os.path.join(ROOT, "tests"))

SETS = [
    ("TTAGGG TCAGGG TGAGGG TTGGGG CTAGGG TTAGGC GGGTTA TTTAGG TTAGGA", "TTCGGG"),  # MANY[0]
    ("TTAGGG", ("ACCCTG" * 6)[:33] + " TGAGGG"),                                  # LONG_TVR[1]
]

code = ("import sys; sys.path.insert(0, %r); from nanotel_amd.api import jit_prebuild; "
        "jit_prebuild(sys.argv[1], sys.argv[2] or None)" % os.path.join(ROOT, "telomere-analyzer_amd"))
procs = [subprocess.Popen([sys.executable, "-c", code, p, t or ""]) for p, t in SETS]
sys.exit(max(p.wait() for p in procs))
