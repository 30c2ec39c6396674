"""End-to-end throughput: FASTQ(.gz) file -> summary.csv through the driver
("End-to-end (file -> summary.csv) Gbases/s is reported
separately").  This is the host-buffer path -- C++ reader, host 2-bit packer,
pageable upload over PCIe, scan + call, rows back, serials, CSV -- not the
bench.py metric (device-resident inputs).

Synthetic Nanopore-like reads (uniform ACGT, half of them with a 1-15 kb
(TTAGGG)n tract at the left edge, 2 % substitutions) are written once with
numpy, then the driver runs over them with NanoTel's default nrec (10,000) unless --nrec says otherwise.
Timed without and with the per-read reads/<serial>.fasta.gz writes, and with
--plots also with the three single-read plots per telomeric read.

    python tools/e2e_bench.py [--reads 8000] [--read_len 50000] [--nrec 10000] [--gz] [--parts 1] [--plots] [--dir /tmp/e2e]
"""
import argparse
import gzip
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "telomere-analyzer_amd"))


def _pool(L, seed, k=512):
    """k distinct synthetic FASTQ bodies (sequence + quality lines) of length L."""
    rng = np.random.default_rng(seed)
    acgt = np.frombuffer(b"ACGT", np.uint8)
    unit = np.frombuffer(b"TTAGGG", np.uint8)
    out = []
    for _ in range(k):
        s = acgt[rng.integers(0, 4, L)]
        if rng.random() < 0.5:
            t = min(L, int(rng.integers(1000, 15001)))
            tract = np.resize(unit, t)
            sub = rng.random(t) < 0.02
            tract[sub] = acgt[rng.integers(0, 4, int(sub.sum()))]
            s[:t] = tract
        out.append(b"\n" + s.tobytes() + b"\n+\n" + b"I" * L + b"\n")
    return out


def _write_part(args):
    name, r0, r1, L, gz, seed = args
    pool = _pool(L, seed)
    op = (lambda p, m: gzip.open(p, m, compresslevel=1)) if gz else open
    with op(name, "wb") as f:
        buf = []
        for r in range(r0, r1):
            buf.append(b"@read_%d" % r + pool[r % len(pool)])
            if len(buf) == 256:
                f.write(b"".join(buf))
                buf = []
        f.write(b"".join(buf))


def write_input(path, n, L, gz, seed=20260501, parts=1):
    """One file, or with parts > 1 a run directory of `parts` files (as a
    sequencer writes them: fastq_pass/part_000.fastq.gz, ...).  The reads
    cycle through a pool of 512 synthetic ones (names stay unique); the parts
    are written by parallel processes."""
    if parts > 1:
        os.makedirs(path, exist_ok=True)
        names = [os.path.join(path, "part_%03d.fastq%s" % (k, ".gz" if gz else "")) for k in range(parts)]
    else:
        names = [path]
    per = (n + len(names) - 1) // len(names)
    jobs = [(nm, k * per, min(n, (k + 1) * per), L, gz, seed) for k, nm in enumerate(names)]
    if len(jobs) > 1:
        import multiprocessing as mp
        with mp.get_context("spawn").Pool(min(16, len(jobs))) as pool:
            pool.map(_write_part, jobs)
    else:
        _write_part(jobs[0])


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reads", type=int, default=8000)
    ap.add_argument("--read_len", type=int, default=50000)
    ap.add_argument("--nrec", type=int, default=10000)
    ap.add_argument("--gz", action="store_true")
    ap.add_argument("--plots", action="store_true", help="also time a run with the single-read plots")
    ap.add_argument("--parts", type=int, default=1, help="write the input as a directory of this many files")
    ap.add_argument("--dir", default="/tmp/nt_e2e")
    ap.add_argument("--profile", default="", help="cProfile the summary-only run into this file (text)")
    ap.add_argument("--no-reads-run", action="store_true", help="skip the run that writes reads/*.fasta.gz")
    ap.add_argument("--cleanup", action="store_true", help="delete the input and outputs at the end")
    ap.add_argument("--gzip-levels", default="6",
                    help="gzip levels of the reads/*.fasta.gz runs (comma separated; 6 = R's gzfile default)")
    a = ap.parse_args()
    os.makedirs(a.dir, exist_ok=True)
    inp = os.path.join(a.dir, "run" if a.parts > 1 else "reads.fastq" + (".gz" if a.gz else ""))
    t = time.perf_counter()
    write_input(inp, a.reads, a.read_len, a.gz, parts=a.parts)
    gen_s = time.perf_counter() - t
    print(f"# input written in {gen_s:.1f} s", file=sys.stderr, flush=True)
    from nanotel_amd import driver
    bases = a.reads * a.read_len
    size = (sum(os.path.getsize(os.path.join(inp, f)) for f in os.listdir(inp)) if os.path.isdir(inp)
            else os.path.getsize(inp))
    out = {"input": os.path.basename(inp), "parts": a.parts, "gz": a.gz, "reads": a.reads, "nrec": a.nrec,
           "read_len": a.read_len, "bases": bases, "input_bytes": size, "generate_s": round(gen_s, 2)}
    # warm-up (hiprtc specialisation, device buffers) on a small prefix-free run
    warm = os.path.join(a.dir, "warm.fastq")
    write_input(warm, min(a.reads, 4000), a.read_len, False, seed=7)
    driver.run(warm, os.path.join(a.dir, "warm"), "TTAGGG", fmt="fastq", nrec=10000, write_reads=False,
               plot=False, log=lambda *x: None)
    print("# warm-up run done", file=sys.stderr, flush=True)
    # the first full-size run also grows the pinned staging and device buffers
    # (a long run pays that once): reported, then the steady-state run
    levels = [int(x) for x in a.gzip_levels.split(",")]
    runs = [("summary_only_first", False, False, None), ("summary_only", False, False, None)]
    if not a.no_reads_run:
        runs += [("with_reads_fasta_gz" + ("" if lv == 6 else f"_level{lv}"), True, False, lv) for lv in levels]
    if a.plots:
        runs.append(("with_reads_and_plots", True, True, levels[0]))
    for key, write_reads, plot, level in runs:
        if level is not None:
            os.environ["NT_GZIP_LEVEL"] = str(level)
        save = os.path.join(a.dir, "out_" + key)
        t = time.perf_counter()
        st = {}
        prof = None
        if a.profile and key == "summary_only":
            import cProfile
            prof = cProfile.Profile()
            prof.enable()
        rows, _ = driver.run(inp, save, "TTAGGG", fmt="fastq", nrec=a.nrec, write_reads=write_reads,
                             plot=plot, log=lambda *x: None, stats=st)
        s = time.perf_counter() - t
        if prof is not None:
            import io as _io
            import pstats
            prof.disable()
            buf = _io.StringIO()
            pstats.Stats(prof, stream=buf).sort_stats("cumulative").print_stats(40)
            open(a.profile, "w").write(buf.getvalue())
        out[key] = {"seconds": round(s, 3), "Gbases_per_s": round(bases / s / 1e9, 3), "rows": len(rows),
                    "phases_s": {k: (round(v, 4) if isinstance(v, float) else v) for k, v in st.items()}}
        print(f"# {key}: {s:.2f} s", file=sys.stderr, flush=True)
    print(json.dumps(out))
    if a.cleanup:
        import shutil
        shutil.rmtree(a.dir, ignore_errors=True)


if __name__ == "__main__":
    main()
