"""The run driver's sharded path on CPU (gloo): chunk rounds, the serial
all_reduce and the row gather must give the same summary.csv / reads files for
1, 2 or 3 ranks.  The GPU scan is replaced by the CPU oracle here (a stand-in
for NanoTel inside the test only); tests/test_gpu_e2e.py runs the real thing."""
import gzip
import os
import socket
import tempfile

import numpy as np
import pytest

import _oracle as O


class OracleNanoTel:
    """Test double of nanotel_amd.NanoTel: same analyze_chunk result layout,
    computed by the oracle (tests only)."""

    def __init__(self, patterns, tvr_patterns=None, subseq_length=100, min_density=0.6,
                 check_right_edge=False, rc=False, legacy_no_ext=False, device=0):
        self.P = O.Patterns(patterns, tvr_patterns)
        self.kw = dict(L=subseq_length, min_density=min_density, right_edge=check_right_edge,
                       legacy_no_ext=legacy_no_ext, want_windows=False, want_hits=False)
        self.rc = rc
        self.n_pass = 3 if tvr_patterns else 2
        self.subseq_length = subseq_length

    def _scan_orientation(self, s):
        s = s.decode() if isinstance(s, bytes) else s
        return O.reverse_complement(s) if self.rc else s

    def filter_chunk(self, ch):
        return np.array([O.filter_read(self._scan_orientation(ch.seq(i)), self.P, self.kw["min_density"],
                                       self.kw["right_edge"]) for i in range(ch.n)], bool)

    def analyze_chunk(self, ch, want_windows=False):
        return self.analyze([ch.seq(i) for i in range(ch.n)], want_windows)

    def analyze_pointers(self, ptrs, lens, want_windows=False):
        import ctypes
        return self.analyze([ctypes.string_at(int(p), int(n)) for p, n in zip(ptrs, lens)], want_windows)

    def analyze(self, seqs, want_windows=False):
        n = len(seqs)
        res = {"start": np.full((n, 3), -1, np.int32), "end": np.full((n, 3), -1, np.int32),
               "density": np.zeros((n, 3)), "telomeric": np.zeros(n, bool),
               "n_windows": np.zeros(n, np.int64), "wins": []}
        kw = dict(self.kw, want_windows=want_windows)
        for i in range(n):
            s = seqs[i].decode() if isinstance(seqs[i], bytes) else seqs[i]
            if self.rc:
                s = O.reverse_complement(s)
            r = O.analyze_read(s, self.P, **kw)
            k = r["n_pass"]
            res["start"][i, :k] = r["start"]
            res["end"][i, :k] = r["end"]
            res["density"][i, :k] = r["density"]
            res["telomeric"][i] = r["telomeric"]
            if want_windows:
                res["n_windows"][i] = len(r["win_counts"][0])
                res["wins"].append(r["win_counts"])
        # the real result's layout: win_off locates a read's counts in win_counts
        res["win_off"], res["win_counts"] = np.arange(n), res["wins"]
        return res

    def window_counts(self, res, read, p):
        return res["win_counts"][int(res["win_off"][read])][p]

    def close(self):
        pass


def _make_input(d, rc=False):
    rng = np.random.default_rng(5)
    names, seqs = O.read_fasta(os.path.join(os.path.dirname(__file__), "golden", "sample.fasta"))
    # under --rc the input holds reverse-complemented telomeric reads, so the
    # first chunk has rows (a first chunk without rows makes every later
    # serial -Inf in the reference: max(numeric(0)) + 1, see test_shard.py)
    recs = [(n, O.reverse_complement(s) if rc else s) for n, s in zip(names, seqs)]
    for i in range(21):
        n = int(rng.integers(200, 4000))
        s = list(rng.choice(list("ACGT"), n))
        if i % 3 != 2:
            t = int(rng.integers(150, min(n, 1500)))
            s[:t] = list(("TTAGGG" * (t // 6 + 1))[:t])
        s = "".join(s)
        recs.append((f"syn_{i} extra", O.reverse_complement(s) if rc else s))
    os.makedirs(os.path.join(d, "in", "sub"))
    with open(os.path.join(d, "in", "a.fasta"), "w") as f:
        for n, s in recs[:13]:
            f.write(f">{n}\n" + "\n".join(s[i:i + 80] for i in range(0, len(s), 80)) + "\n")
    with gzip.open(os.path.join(d, "in", "sub", "b.fasta.gz"), "wt") as f:
        for n, s in recs[13:]:
            f.write(f">{n}\n{s}\n")
    return os.path.join(d, "in")


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _rank_main(rank, world, port, inp, out, rc, use_filter=False, g=1, fmt="fasta", nrec=3, stats_dir=None):
    """One rank of a driver run (g: chunks per block, NT_GROUP_CHUNKS -- 1 deals
    the few chunks of these small inputs over every rank)."""
    import json
    import torch.distributed as dist
    from nanotel_amd import driver
    driver.NanoTel = OracleNanoTel
    if g is not None:
        os.environ["NT_GROUP_CHUNKS"] = str(g)
    if world > 1:
        os.environ["MASTER_ADDR"] = "127.0.0.1"
        os.environ["MASTER_PORT"] = str(port)
        dist.init_process_group("gloo", rank=rank, world_size=world)
    st = {}
    driver.run(inp, out, "TTAGGG", fmt=fmt, nrec=nrec, rc=rc, use_filter=use_filter, analysis=True,
               log=lambda *a: None, stats=st)
    if stats_dir is not None:
        with open(os.path.join(stats_dir, f"stats_{world}_{rank}.json"), "w") as f:
            json.dump({k: v for k, v in st.items() if isinstance(v, (int, float, str))}, f)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


def _outputs(out):
    files = {}
    for root, _, fs in os.walk(out):
        for f in fs:
            p = os.path.join(root, f)
            rel = os.path.relpath(p, out)
            if f == "run.log":
                continue
            files[rel] = gzip.open(p).read() if f.endswith(".gz") else open(p, "rb").read()
    return files


def _forced_one_rank(rank, port, inp, out):
    # a one-rank process group whose collectives run anyway (NT_DIST_FORCE=1):
    # the path RCCL takes on a one-GPU box (test_gpu_e2e's nccl cases)
    import torch.distributed as dist
    from nanotel_amd import driver, shard
    os.environ["NT_DIST_FORCE"] = "1"
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=0, world_size=1)
    calls = []
    real = dist.all_reduce
    dist.all_reduce = lambda *a, **k: (calls.append(1), real(*a, **k))[1]
    try:
        driver.NanoTel = OracleNanoTel
        driver.run(inp, out, "TTAGGG", fmt="fasta", nrec=3, log=lambda *a: None)
    finally:
        dist.all_reduce = real
    assert shard._collective() and len(calls) >= 2  # the per-round exchange and the end-of-run flags
    dist.destroy_process_group()


def test_forced_collectives_on_one_rank():
    import torch.multiprocessing as mp
    with tempfile.TemporaryDirectory() as d:
        inp = _make_input(d, False)
        _rank_main(0, 1, 0, inp, os.path.join(d, "plain"), False)
        mp.spawn(_forced_one_rank, args=(_free_port(), inp, os.path.join(d, "forced")), nprocs=1, join=True)
        a, b = _outputs(os.path.join(d, "plain")), _outputs(os.path.join(d, "forced"))
        for k in ("in_filtered_sorted_summary.csv", "in_results.txt", "in_telomere_plot.png"):
            a.pop(k, None)
        assert a == b and len(a["in_summary.csv"].splitlines()) > 5


@pytest.mark.parametrize("rc", [False, True])
def test_sharded_driver_matches_single_process(rc):
    import torch.multiprocessing as mp
    with tempfile.TemporaryDirectory() as d:
        inp = _make_input(d, rc)
        res = {}
        for world in (1, 2, 3):
            out = os.path.join(d, f"out{world}")
            if world == 1:
                _rank_main(0, 1, 0, inp, out, rc)
            else:
                mp.spawn(_rank_main, args=(world, _free_port(), inp, out, rc), nprocs=world, join=True)
            res[world] = _outputs(out)
        assert res[1] == res[2] == res[3]
        summary = res[1]["in_summary.csv"].decode().splitlines()
        assert summary[0].startswith("Serial,sequence_ID,")
        assert len(summary) > 5
        # Serial values are 1..rows in the reference's chunk/group order
        assert [int(line.split(",")[0]) for line in summary[1:]] == sorted(
            int(line.split(",")[0]) for line in summary[1:])
        assert res[1]["reads_ids.txt"].decode().splitlines() == [line.split(",")[1] for line in summary[1:]]
        # --analysis outputs (rank 0) agree across world sizes too and follow analysis.analyze
        from nanotel_amd import analysis
        assert "in_filtered_sorted_summary.csv" in res[1] and "in_results.txt" in res[1]
        fs = res[1]["in_filtered_sorted_summary.csv"].decode().splitlines()
        assert fs[0].endswith(",TelLenMM_RunningMed,SeqLen_minus_RunMed")
        assert res[1]["in_results.txt"].decode().splitlines()[2].endswith(f": {len(fs) - 1}")
        lens = [int(line.split(",")[2]) for line in fs[1:]]
        assert lens == sorted(lens, reverse=True) and analysis.MAX_START_MM == 134


def _filter_input(d):
    """Chunks of 3 (nrec=3) for --use_filter: chunk 1 loses every read to the
    filter (short, or no telomeric edge), later chunks keep some."""
    rng = np.random.default_rng(9)

    def read(n, edge_tract):
        s = list(rng.choice(list("ACGT"), n))
        if edge_tract:
            t = int(rng.integers(400, 1500))
            s[:t] = list(("TTAGGG" * (t // 6 + 1))[:t])
        return "".join(s)

    recs = [("short_telo", read(900, True)), ("plain_a", read(3000, False)), ("plain_b", read(1500, False))]
    for i in range(16):
        recs.append((f"r{i}", read(int(rng.integers(1000, 5000)), i % 4 != 3)))
    recs += [("plain_c", read(2000, False)), ("plain_d", read(2500, False)), ("plain_e", read(800, True))]
    recs += [("last", read(3000, True))]
    os.makedirs(os.path.join(d, "in"))
    with open(os.path.join(d, "in", "a.fasta"), "w") as f:
        for n, s in recs:
            f.write(f">{n}\n{s}\n")
    return os.path.join(d, "in"), recs


def _reference_filter_rows(recs, nrec=3):
    """run_future_worker_chuncks with use_filter (NanoTel.R:2209-2258) over the
    oracle: a chunk the filter empties is skipped (`next`) without touching
    serial_start; otherwise the kept reads are grouped and numbered as usual
    and serial_start = max(all Serial) + 1."""
    P = O.Patterns("TTAGGG")
    serial_start, mx, rows = 1.0, -np.inf, []
    for c in range(0, len(recs), nrec):
        chunk = recs[c:c + nrec]
        kept = [(n, s) for n, s in chunk if O.filter_read(s, P)]
        if not kept:
            continue
        telo = np.array([O.analyze_read(s, P)["telomeric"] for _, s in kept], np.uint8)
        ser, order, serial_start, mx = O.assign_serials(telo, serial_start, mx)
        rows += [(float(ser[j]), kept[j][0]) for j in order]
    return rows


def test_use_filter_driver_matches_reference_flow():
    import torch.multiprocessing as mp
    with tempfile.TemporaryDirectory() as d:
        inp, recs = _filter_input(d)
        expect = _reference_filter_rows(recs)
        assert 5 < len(expect) < 19
        res = {}
        for world in (1, 2):
            out = os.path.join(d, f"out{world}")
            if world == 1:
                _rank_main(0, 1, 0, inp, out, False, True)
            else:
                mp.spawn(_rank_main, args=(world, _free_port(), inp, out, False, True), nprocs=world, join=True)
            res[world] = _outputs(out)
        assert res[1] == res[2]
        lines = res[1]["in_summary.csv"].decode().splitlines()[1:]
        got = [(float(x.split(",")[0]), x.split(",")[1]) for x in lines]
        assert got == expect
        assert got[0][0] == 1.0  # the emptied first chunk left serial_start at 1


def test_filter_oracle_edges():
    P = O.Patterns("TTAGGG")
    tel = "TTAGGG" * 16  # 96 of 200 covered = 0.48 = 0.8 * 0.6
    assert O.filter_read("A" * 70 + tel + "C" * 1000, P)
    assert not O.filter_read("A" * 70 + tel[:-6] + "C" * 1000, P)
    assert not O.filter_read("A" * 70 + tel + "C" * 763, P)  # 999 bases: dropped
    assert not O.filter_read("A" * 71 + tel + "C" * 1000, P, min_density=0.61)
    s = "C" * 1000 + tel + "A" * 70  # right edge sub-read [n-269, n-70]
    assert O.filter_read(s, P, right_edge=True) and not O.filter_read(s, P)
    # fixed=FALSE: a subject N matches any pattern letter
    assert O.filter_read("A" * 70 + "N" * 96 + "C" * 1000, P)


def _inf_input(d):
    """Chunk 1 (nrec=3) has no telomeric read: the reference's serial_start
    becomes max(numeric(0)) + 1 = -Inf and every later row is -Inf, so all
    telomeric reads name reads/-Inf.fasta.gz (NanoTel.R:1871, 2258)."""
    rng = np.random.default_rng(21)

    def read(n, tract):
        s = list(rng.choice(list("ACGT"), n))
        if tract:
            t = int(rng.integers(300, min(n, 1500)))
            s[:t] = list(("TTAGGG" * (t // 6 + 1))[:t])
        return "".join(s)

    recs = [(f"plain{i}", read(2000, False)) for i in range(3)]
    recs += [(f"t{i}", read(int(rng.integers(1500, 4000)), i % 3 != 1)) for i in range(14)]
    os.makedirs(os.path.join(d, "in"))
    with open(os.path.join(d, "in", "a.fasta"), "w") as f:
        for n, s in recs:
            f.write(f">{n}\n{s}\n")
    return os.path.join(d, "in"), recs


def test_inf_serials_write_the_last_read_once():
    import torch.multiprocessing as mp
    with tempfile.TemporaryDirectory() as d:
        inp, recs = _inf_input(d)
        P = O.Patterns("TTAGGG")
        telo = [n for n, s in recs if O.analyze_read(s, P)["telomeric"]]
        assert telo and not any(n.startswith("plain") for n in telo)
        res = {}
        for world in (1, 2, 3):
            out = os.path.join(d, f"out{world}")
            if world == 1:
                _rank_main(0, 1, 0, inp, out, False)
            else:
                mp.spawn(_rank_main, args=(world, _free_port(), inp, out, False), nprocs=world, join=True)
            res[world] = _outputs(out)
        assert res[1] == res[2] == res[3]
        lines = res[1]["in_summary.csv"].decode().splitlines()[1:]
        assert len(lines) == len(telo) and all(x.startswith("-Inf,") for x in lines)
        reads = sorted(k for k in res[1] if k.startswith("reads" + os.sep))
        assert reads == [os.path.join("reads", "-Inf.fasta.gz")]
        # the row written last in the stream: the last telomeric read in row order
        last = lines[-1].split(",")[1]
        assert res[1][reads[0]].decode().splitlines()[0] == ">" + last
        seq = dict(recs)[last]
        assert "".join(res[1][reads[0]].decode().splitlines()[1:]) == seq


class FailingNanoTel(OracleNanoTel):
    """Raises on the device call it makes on rank 1 of a 2-rank run."""

    def analyze_pointers(self, ptrs, lens, want_windows=False):
        import torch.distributed as dist
        if dist.is_initialized() and dist.get_rank() == 1:
            raise RuntimeError("injected scan failure")
        return super().analyze_pointers(ptrs, lens, want_windows)


def _failing_rank(rank, world, port, inp, out, q):
    import torch.distributed as dist
    from nanotel_amd import driver
    driver.NanoTel = FailingNanoTel
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    os.environ["NT_GROUP_CHUNKS"] = "1"
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        driver.run(inp, out, "TTAGGG", fmt="fasta", nrec=3, log=lambda *a: None, plot=False)
        q.put((rank, "ok"))
    except Exception as ex:  # noqa: BLE001
        q.put((rank, str(ex)))
    dist.destroy_process_group()


@pytest.mark.timeout(180)
def test_rank_failure_stops_every_rank():
    """A rank that fails inside a chunk round publishes the error flag with the
    serial all_reduce: every rank raises at that round (the reference stops at
    the first error) instead of waiting in the next collective."""
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    with tempfile.TemporaryDirectory() as d:
        inp = _make_input(d)
        q = ctx.Queue()
        port = _free_port()
        ps = [ctx.Process(target=_failing_rank, args=(r, 2, port, inp, os.path.join(d, "o"), q)) for r in range(2)]
        for p in ps:
            p.start()
        for p in ps:
            p.join(150)
        alive = [p.is_alive() for p in ps]
        for p in ps:
            if p.is_alive():
                p.kill()
        assert not any(alive)
        got = dict(q.get(timeout=5) for _ in range(2))
        assert got[1] == "injected scan failure"
        assert "another rank failed" in got[0]


def _shard_records(n=61, seed=31):
    rng = np.random.default_rng(seed)
    recs = []
    for i in range(n):
        m = int(rng.integers(150, 3000))
        s = list(rng.choice(list("ACGT"), m))
        if i % 3 != 2:
            t = int(rng.integers(150, min(m, 1500)))
            s[:t] = list(("TTAGGG" * (t // 6 + 1))[:t])
        recs.append((f"rd{i} ch={i % 7}", "".join(s)))
    return recs, rng


def _write_shard_inputs(d):
    """The three input shapes of a sharded run: one plain FASTQ (CRLF, quality
    lines that start with '@' or '+', a blank line between records), one
    wrapped FASTA, and a run directory of 16 fastq.gz parts (two empty)."""
    recs, rng = _shard_records()
    qual = lambda s: "".join(rng.choice(list("@+I#5"), len(s)))  # noqa: E731
    fq = os.path.join(d, "reads.fastq")
    with open(fq, "w", newline="") as f:
        for i, (n, s) in enumerate(recs):
            f.write(f"@{n}\r\n{s}\r\n+\r\n{qual(s)}\r\n" + ("\n" if i % 5 == 4 else ""))
    fa = os.path.join(d, "reads.fasta")
    with open(fa, "w") as f:
        for n, s in recs:
            f.write(f">{n}\n" + "\n".join(s[i:i + 70] for i in range(0, len(s), 70)) + "\n")
    run = os.path.join(d, "run")
    os.makedirs(run)
    cuts = np.sort(np.concatenate([[0, 0, len(recs), len(recs)], rng.integers(0, len(recs), 13)]))
    for p in range(16):
        with gzip.open(os.path.join(run, f"part_{p:02d}.fastq.gz"), "wt") as f:
            for n, s in recs[cuts[p]:cuts[p + 1]]:
                f.write(f"@{n}\n{s}\n+\n{qual(s)}\n")
    return {"fastq": (fq, "fastq", "range"), "fasta": (fa, "fasta", "range"), "run": (run, "fastq", "files")}


def _expected_inflate(run, world, g, nrec):
    """Bytes each rank of a sharded run over a directory of fastq.gz parts
    inflates: its count-pass parts (p = rank mod world) and every part that
    holds a record of its blocks (blocks of g chunks dealt round-robin)."""
    parts = sorted(os.listdir(run))
    data = [gzip.open(os.path.join(run, p), "rb").read() for p in parts]
    counts = [x.count(b"\n") // 4 for x in data]
    first = np.concatenate([[0], np.cumsum(counts)])
    total = int(first[-1])
    n_chunks = -(-total // nrec)
    out = []
    for r in range(world):
        b = sum(len(data[p]) for p in range(r, len(parts), world))
        need = set()
        for k0 in range(r * g, n_chunks, g * world):
            r0, r1 = k0 * nrec, min((k0 + g) * nrec, total) - 1
            f0 = int(np.searchsorted(first, r0, side="right")) - 1
            f1 = int(np.searchsorted(first, r1, side="right")) - 1
            need.update(range(f0, max(f0, f1) + 1))
        out.append(b + sum(len(data[p]) for p in need))
    return out


@pytest.mark.timeout(600)
def test_sharded_ingest_outputs_identical_across_world_sizes():
    """Every rank reads only its own chunks: for a plain FASTQ,
    a wrapped FASTA and a 16-part fastq.gz run directory, world 1/2/3/8 write
    byte-identical outputs, the plan is sharded ("range" / "files"), and each
    rank parses about 2/N of the input bytes (its index share plus its chunks),
    not the whole stream."""
    import json
    import torch.multiprocessing as mp
    with tempfile.TemporaryDirectory() as d:
        for key, (inp, fmt, mode) in _write_shard_inputs(d).items():
            res = {}
            g = 1 if mode == "range" else 2  # a block of the run directory spans about 2 parts
            for world in (1, 2, 3, 8):
                out = os.path.join(d, f"{key}_out{world}")
                sd = os.path.join(d, f"{key}_stats")
                os.makedirs(sd, exist_ok=True)
                if world == 1:
                    _rank_main(0, 1, 0, inp, out, False, False, g, fmt, 4, sd)
                else:
                    mp.spawn(_rank_main, args=(world, _free_port(), inp, out, False, False, g, fmt, 4, sd),
                             nprocs=world, join=True)
                res[world] = _outputs(out)
                st = [json.load(open(os.path.join(sd, f"stats_{world}_{r}.json"))) for r in range(world)]
                if world > 1:
                    assert all(s["ingest"] == mode for s in st), (key, world, st[0])
                    size = sum(os.path.getsize(os.path.join(r, f)) for r, _, fs in os.walk(inp) for f in fs) \
                        if os.path.isdir(inp) else os.path.getsize(inp)
                    if mode == "range":
                        # every rank's parse: its 1/N index share + its chunks
                        assert max(s["bytes_parsed"] for s in st) < size * (2.0 / world + 0.25), (key, world, st)
                        assert sum(s["bytes_parsed"] for s in st) < 2.2 * size
                    else:
                        # gzip parts: the count pass inflates parts p = r (mod N),
                        # the chunk reads exactly the parts the rank's blocks touch
                        assert [s["bytes_inflated"] for s in st] == _expected_inflate(inp, world, g, 4), (key, world)
            assert res[1] == res[2] == res[3] == res[8], key
            summary = res[1][f"{os.path.basename(inp)}_summary.csv"].decode().splitlines()
            assert len(summary) > 20


@pytest.mark.parametrize("g", [1, 2, None])
def test_block_ownership_world2(g):
    """Blocks of g chunks (None: the default, ceil(65536 / nrec) capped at 16)
    give the files of a single process."""
    import torch.multiprocessing as mp
    with tempfile.TemporaryDirectory() as d:
        inp = _make_input(d, False)
        _rank_main(0, 1, 0, inp, os.path.join(d, "one"), False)
        mp.spawn(_rank_main, args=(2, _free_port(), inp, os.path.join(d, "two"), False, False, g),
                 nprocs=2, join=True)
        assert _outputs(os.path.join(d, "one")) == _outputs(os.path.join(d, "two"))


def test_dist_backend_choice():
    """RCCL by default when every local rank has its own GPU; gloo when ranks
    share one (explicit --device, more local ranks than GPUs) or run alone;
    NT_DIST_BACKEND overrides."""
    from nanotel_amd.cli import dist_backend
    assert dist_backend(8, 8, None, 8, env={}) == "nccl"
    assert dist_backend(2, 2, None, 1, env={}) == "gloo"
    assert dist_backend(2, 2, 0, 8, env={}) == "gloo"
    assert dist_backend(1, 1, None, 8, env={}) == "gloo"
    assert dist_backend(8, 8, None, 8, env={"NT_DIST_BACKEND": "gloo"}) == "gloo"
    assert dist_backend(1, 1, None, 1, env={"NT_DIST_BACKEND": "nccl"}) == "nccl"


class FastNanoTel:
    """Test double of nanotel_amd.NanoTel for the row stream at scale: rows
    computed from the read lengths alone (vectorised), so that a gloo run of
    10^6 rows takes seconds.  Two thirds of the reads are telomeric; pass 1
    is NA for one read in eleven."""

    def __init__(self, patterns, tvr_patterns=None, subseq_length=100, min_density=0.6,
                 check_right_edge=False, rc=False, legacy_no_ext=False, device=0):
        self.n_pass = 3 if tvr_patterns else 2
        self.subseq_length = subseq_length

    def analyze_pointers(self, ptrs, lens, want_windows=False):
        n = lens.size
        ln = lens.astype(np.int64)
        st = np.full((n, 3), -1, np.int32)
        en = np.full((n, 3), -1, np.int32)
        st[:, :2] = (1 + ln % 7)[:, None]
        en[:, :2] = (ln - ln % 5)[:, None]
        na = ln % 11 == 0
        st[na, 0] = en[na, 0] = -1
        dens = np.zeros((n, 3))
        dens[:, :2] = ((ln % 97) / 97.0)[:, None]
        return {"start": st, "end": en, "density": dens, "telomeric": ln % 3 != 0}

    def close(self):
        pass


def _big_rank(rank, world, port, inp, out, stats_dir):
    import json
    import torch.distributed as dist
    from nanotel_amd import driver
    driver.NanoTel = FastNanoTel
    if world > 1:
        os.environ["MASTER_ADDR"] = "127.0.0.1"
        os.environ["MASTER_PORT"] = str(port)
        dist.init_process_group("gloo", rank=rank, world_size=world)
    st = {}
    driver.run(inp, out, "TTAGGG", fmt="fasta", nrec=2000, write_reads=False, plot=False,
               log=lambda *a: None, stats=st)
    with open(os.path.join(stats_dir, f"big_{world}_{rank}.json"), "w") as f:
        json.dump({k: v for k, v in st.items() if isinstance(v, (int, float, str))}, f)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


@pytest.mark.timeout(900)
def test_row_stream_million_rows_identical_across_world_sizes(tmp_path):
    """the rows go to rank 0 group round by group round (no
    end-of-run gather of every row).  1.2 M reads, >= 10^6 rows: world 2 and 8
    (gloo) write summary.csv / reads_ids.txt byte-identical to world 1, rank 0
    never receives more than one round's rows at a time, and every rank's peak
    RSS is recorded (stats JSON beside the outputs)."""
    import json
    import torch.multiprocessing as mp
    rng = np.random.default_rng(123)
    n = 1_560_000
    lens = rng.integers(40, 130, n)
    inp = tmp_path / "big.fasta"
    with open(inp, "wb") as f:
        seq = b"ACGT" * 40
        f.write(b"".join(b">r%d x\n%s\n" % (i, seq[:int(k)]) for i, k in enumerate(lens)))
    n_rows = int((lens % 3 != 0).sum())
    assert n_rows >= 1_000_000
    outs, st = {}, {}
    for world in (1, 2, 8):
        out = tmp_path / f"out{world}"
        if world == 1:
            _big_rank(0, 1, 0, str(inp), str(out), str(tmp_path))
        else:
            mp.start_processes(_big_rank, args=(world, _free_port(), str(inp), str(out), str(tmp_path)),
                               nprocs=world, join=True, start_method="spawn")
        outs[world] = {f: (out / f).read_bytes() for f in ("big.fasta_summary.csv", "reads_ids.txt")}
        st[world] = [json.load(open(tmp_path / f"big_{world}_{r}.json")) for r in range(world)]
    assert outs[1]["big.fasta_summary.csv"].count(b"\n") == n_rows + 1
    for world in (2, 8):
        assert outs[world] == outs[1], world
    total = sum(len(v) for v in outs[1].values())
    for world in (1, 2, 8):
        s0 = st[world][0]
        assert s0["rows_rounds"] >= 3, s0  # several rounds ...
        assert s0["rows_max_round_bytes"] <= total // 2, s0  # ... none holding the run's rows
        print(f"world {world}: rank-0 peak RSS {s0['peak_rss_kb'] / 1024:.0f} MiB, "
              f"{s0['rows_rounds']} rounds, at most {s0['rows_max_round_bytes'] / 2**20:.1f} MiB of rows a round "
              f"(of {total / 2**20:.1f} MiB); other ranks' peak RSS "
              f"{[round(x['peak_rss_kb'] / 1024) for x in st[world][1:]]} MiB")
