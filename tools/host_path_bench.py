"""Host-buffer rate of nt_analyze_host (PCIe-inclusive, not the
bench.py metric): ASCII reads already in host memory -> host 2-bit packer ->
upload -> scan + call -> rows (+ window counts) back.  Also times the packer
alone (nt_pack_count + nt_pack_reads into host memory).

    python tools/host_path_bench.py [--reads 4000] [--read_len 50000] [--reps 5]
"""
import argparse
import ctypes
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "telomere-analyzer_amd"))


def make_reads(n, L, seed=20260501):
    rng = np.random.default_rng(seed)
    acgt = np.frombuffer(b"ACGT", np.uint8)
    unit = np.frombuffer(b"TTAGGG", np.uint8)
    out = []
    for r in range(n):
        s = acgt[rng.integers(0, 4, L)]
        if r % 2 == 0:
            t = int(rng.integers(1000, 15001))
            s[:t] = np.resize(unit, t)
        out.append(s.tobytes())
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reads", type=int, default=4000)
    ap.add_argument("--read_len", type=int, default=50000)
    ap.add_argument("--reps", type=int, default=5)
    a = ap.parse_args()
    from nanotel_amd import NanoTel, lib
    seqs = make_reads(a.reads, a.read_len)
    bases = a.reads * a.read_len
    n = len(seqs)
    ptrs = (ctypes.c_char_p * n)(*seqs)
    lens = np.array([len(s) for s in seqs], np.uint64)
    L = lib()
    tb, tw, te, ml, bad = (ctypes.c_uint64() for _ in range(5))
    pk = []
    for _ in range(a.reps):
        t = time.perf_counter()
        L.nt_pack_count(ctypes.cast(ptrs, ctypes.c_void_p), lens.ctypes.data, n, 100, ctypes.byref(tb),
                        ctypes.byref(tw), ctypes.byref(te), ctypes.byref(ml), ctypes.byref(bad))
        planes = np.empty(2 * tb.value + 2, np.uint32)
        blk, ln, wo = np.empty(n, np.uint64), np.empty(n, np.uint32), np.empty(n, np.uint64)
        L.nt_pack_reads(ctypes.cast(ptrs, ctypes.c_void_p), lens.ctypes.data, n, 0, 100, planes.ctypes.data,
                        blk.ctypes.data, ln.ctypes.data, wo.ctypes.data, None, None, None)
        pk.append(time.perf_counter() - t)
    out = {"reads": n, "read_len": a.read_len, "bases": bases, "host_cpus": os.cpu_count(), "host_threads": min(16, os.cpu_count() or 1)}
    out["pack_only"] = {"seconds": round(min(pk), 4), "Gbases_per_s": round(bases / min(pk) / 1e9, 2)}
    with NanoTel("TTAGGG") as nt:
        for want in (False, True):
            nt.analyze(seqs[:64], want_windows=want)
            ts = []
            for _ in range(a.reps):
                t = time.perf_counter()
                res = nt.analyze(seqs, want_windows=want)
                ts.append(time.perf_counter() - t)
            key = "analyze_host_with_window_counts" if want else "analyze_host"
            out[key] = {"seconds": round(min(ts), 4), "Gbases_per_s": round(bases / min(ts) / 1e9, 2),
                        "telomeric": int(res["telomeric"].sum())}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
