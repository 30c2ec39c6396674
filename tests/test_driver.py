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

    def analyze_chunk(self, ch):
        n = ch.n
        res = {"start": np.full((n, 3), -1, np.int32), "end": np.full((n, 3), -1, np.int32),
               "density": np.zeros((n, 3)), "telomeric": np.zeros(n, bool)}
        for i in range(n):
            s = ch.seq(i).decode()
            if self.rc:
                s = O.reverse_complement(s)
            r = O.analyze_read(s, self.P, **self.kw)
            k = r["n_pass"]
            res["start"][i, :k] = r["start"]
            res["end"][i, :k] = r["end"]
            res["density"][i, :k] = r["density"]
            res["telomeric"][i] = r["telomeric"]
        return res

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


def _rank_main(rank, world, port, inp, out, rc):
    import torch.distributed as dist
    from nanotel_amd import driver
    driver.NanoTel = OracleNanoTel
    if world > 1:
        os.environ["MASTER_ADDR"] = "127.0.0.1"
        os.environ["MASTER_PORT"] = str(port)
        dist.init_process_group("gloo", rank=rank, world_size=world)
    driver.run(inp, out, "TTAGGG", fmt="fasta", nrec=3, rc=rc, log=lambda *a: None)
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
