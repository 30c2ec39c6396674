"""End to end on the GPU: the command line (python -m nanotel_amd) reading
FASTA/FASTQ(.gz), scanning on the MI355X and writing summary.csv,
reads_ids.txt, reads/<serial>.fasta.gz and the single-read plots.

* Example/sample.fasta in legacy mode (the 2023 code that produced
  Example_output) -> byte-identical summary.csv, reads/*.fasta and
  single_read_plots_adj/read*.eps;
* a multi-file, multi-chunk FASTQ(.gz) input -> the same files as the
  oracle-driven driver (tests/test_driver.py's stand-in).
"""
import gzip
import os
import shutil

import numpy as np
import pytest

import _oracle as O
from test_driver import OracleNanoTel, _make_input, _outputs

pytestmark = pytest.mark.gpu

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def test_cli_example_legacy_byte_identical(tmp_path):
    from nanotel_amd.cli import main
    inp = tmp_path / "sample.fasta"
    shutil.copyfile(os.path.join(GOLD, "sample.fasta"), inp)
    out = tmp_path / "out"
    assert main(["-i", str(inp), "--save_path", str(out), "--format", "fasta", "--patterns", "TTAGGG",
                 "--legacy_no_ext"]) == 0
    assert (out / "sample.fasta_summary.csv").read_bytes() == open(
        os.path.join(GOLD, "example_summary.csv"), "rb").read()
    for i in range(1, 5):
        assert gzip.open(out / "reads" / f"{i}.fasta.gz").read() == open(
            os.path.join(GOLD, "reads", f"{i}.fasta"), "rb").read()
    names, _ = O.read_fasta(os.path.join(GOLD, "sample.fasta"))
    assert (out / "reads_ids.txt").read_text().splitlines() == names
    # the single-read EPS plots from the GPU's window counts: the reference's files byte for byte
    for i in range(1, 5):
        assert (out / "single_read_plots_adj" / f"read{i}.eps").read_bytes() == open(
            os.path.join(GOLD, "eps", f"read{i}.eps"), "rb").read()
        assert (out / "single_read_plots" / f"read{i}.jpeg").stat().st_size > 1000
        assert (out / "single_read_plots_adj" / f"read{i}.jpeg").stat().st_size > 1000


def test_cli_example_current_code(tmp_path):
    # current code (edge extension on): SURVEY §8(c) predicted rows
    from nanotel_amd.cli import main
    inp = tmp_path / "sample.fasta"
    shutil.copyfile(os.path.join(GOLD, "sample.fasta"), inp)
    out = tmp_path / "out"
    assert main(["-i", str(inp), "--save_path", str(out), "--format", "fasta", "--patterns", "TTAGGG"]) == 0
    lines = (out / "sample.fasta_summary.csv").read_text().splitlines()
    assert lines[2].endswith("0.9630518234165067,12070,20405,8336,0.9743309666848716,11251,20405,9155")
    assert lines[3].endswith("0.9837031219320637,49241,59426,10186,0.9906408174959411,48956,59426,10471")
    assert lines[4].endswith("0.9705955437753665,3805,15877,12073,0.9874927524227616,3805,15877,12073")


@pytest.mark.parametrize("rc", [False, True])
def test_driver_gpu_matches_oracle_driver(tmp_path, rc):
    from nanotel_amd import driver
    inp = _make_input(str(tmp_path), rc)
    gpu_out, ora_out = str(tmp_path / "gpu"), str(tmp_path / "ora")
    driver.run(inp, gpu_out, "TTAGGG", fmt="fasta", nrec=4, rc=rc, log=lambda *a: None)
    real = driver.NanoTel
    try:
        driver.NanoTel = OracleNanoTel
        driver.run(inp, ora_out, "TTAGGG", fmt="fasta", nrec=4, rc=rc, log=lambda *a: None)
    finally:
        driver.NanoTel = real
    a, b = _outputs(gpu_out), _outputs(ora_out)
    assert a == b
    assert len(a["in_summary.csv"].splitlines()) > 5
    assert np.all([k.endswith((".fasta.gz", ".eps", ".jpeg")) or k in ("in_summary.csv", "reads_ids.txt") for k in a])
    assert any(k.endswith(".eps") for k in a)  # the plots (window counts from the GPU) match too


def test_driver_use_filter_gpu_matches_oracle_driver(tmp_path):
    from nanotel_amd import driver
    from test_driver import _filter_input
    inp, _ = _filter_input(str(tmp_path))
    gpu_out, ora_out = str(tmp_path / "gpu"), str(tmp_path / "ora")
    driver.run(inp, gpu_out, "TTAGGG", fmt="fasta", nrec=3, use_filter=True, log=lambda *a: None)
    real = driver.NanoTel
    try:
        driver.NanoTel = OracleNanoTel
        driver.run(inp, ora_out, "TTAGGG", fmt="fasta", nrec=3, use_filter=True, log=lambda *a: None)
    finally:
        driver.NanoTel = real
    a, b = _outputs(gpu_out), _outputs(ora_out)
    assert a == b
    assert len(a["in_summary.csv"].splitlines()) > 5


def test_cli_two_ranks_match_one(tmp_path):
    """The command line under torch.distributed.run with 2 ranks (sharded
    ingest: the ranks count the input's files between them and each reads only
    its blocks of chunks -- one chunk a block here, NT_GROUP_CHUNKS; one serial
    all_reduce per group, rows gathered to rank 0) writes the same files as one
    process.  Both ranks use GPU 0 here, so the collectives run on gloo
    (NT_DIST_BACKEND); on a node each rank has its GPU and RCCL (the default,
    cli.dist_backend)."""
    import socket
    import subprocess
    import sys
    inp = _make_input(str(tmp_path), False)
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, PYTHONPATH=os.path.join(root, "telomere-analyzer_amd"), NT_DIST_BACKEND="gloo",
               HSA_ENABLE_IPC_MODE_LEGACY="0", NT_GROUP_CHUNKS="1")
    args = ["-i", inp, "--format", "fasta", "--patterns", "TTAGGG", "-n", "4", "--device", "0"]
    one = str(tmp_path / "one")
    subprocess.run([sys.executable, "-m", "nanotel_amd", "--save_path", one] + args, env=env, check=True,
                   timeout=120)
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    two = str(tmp_path / "two")
    subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
                    "--master-addr", "127.0.0.1", "--master-port", str(port), "-m", "nanotel_amd",
                    "--save_path", two] + args, env=env, check=True, timeout=180)
    a, b = _outputs(one), _outputs(two)
    assert a == b and len(a["in_summary.csv"].splitlines()) > 5


@pytest.mark.parametrize("launcher", ["self", "torchrun"])
def test_bench_two_ranks(launcher):
    """bench.py --gpus 2 (weak scaling: each rank scans its own reads,
    max-over-ranks time, whole-job value): the driver's N-GPU measurement path,
    rehearsed on one GPU (both ranks on GPU 0, host collectives,
    NT_BENCH_BACKEND=gloo).  "self": run with no launcher, bench.py starts its
    own 2 ranks; "torchrun": under torch.distributed.run, as the driver does."""
    import json
    import socket
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, NT_BENCH_BACKEND="gloo", HSA_ENABLE_IPC_MODE_LEGACY="0")
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK"):
        env.pop(k, None)
    args = ["--gpus", "2", "--steps", "3", "--warmup", "1", "--config", "c10k", "--reads", "20000",
            "--no-cpu-baseline"]
    cmd = [sys.executable, os.path.join(root, "bench.py")] + args
    if launcher == "torchrun":
        s = socket.socket()
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
        s.close()
        cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
               "--master-addr", "127.0.0.1", "--master-port", str(port)] + cmd[1:]
    r = subprocess.run(cmd, env=env, check=True, timeout=240, capture_output=True, text=True)
    lines = [x for x in r.stdout.splitlines() if x.startswith("{")]
    assert len(lines) == 1, r.stdout  # rank 0 prints the one JSON line
    d = json.loads(lines[0])
    assert d["n_gpus"] == 2 and d["scaling"] == "weak" and d["value"] > 0
    # value = bases of both ranks / the slower rank's time
    assert abs(d["value"] - 2 * 20000 * 10000 * 3 / (d["ms_per_step"] * 3 / 1e3) / 1e9) < 0.01 * d["value"]



def _port():
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_cli_rccl_one_rank_matches_plain(tmp_path):
    """The driver's RCCL path (NT_DIST_BACKEND=nccl: the per-round all_reduce,
    the held-chunk max and the failure flags on device tensors, the rows by
    gather_object) on the one GPU of this box: a one-rank RCCL group whose
    collectives run anyway (NT_DIST_FORCE=1) writes the files of a plain run."""
    import subprocess
    import sys
    inp = _make_input(str(tmp_path), False)
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, PYTHONPATH=os.path.join(root, "telomere-analyzer_amd"), HSA_ENABLE_IPC_MODE_LEGACY="0")
    args = ["-i", inp, "--format", "fasta", "--patterns", "TTAGGG", "-n", "4", "--device", "0"]
    one = str(tmp_path / "one")
    subprocess.run([sys.executable, "-m", "nanotel_amd", "--save_path", one] + args, env=env, check=True,
                   timeout=120)
    rccl = str(tmp_path / "rccl")
    env.update(NT_DIST_BACKEND="nccl", NT_DIST_FORCE="1")
    subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "1",
                    "--master-addr", "127.0.0.1", "--master-port", str(_port()), "-m", "nanotel_amd",
                    "--save_path", rccl] + args, env=env, check=True, timeout=180)
    a, b = _outputs(one), _outputs(rccl)
    assert a == b and len(a["in_summary.csv"].splitlines()) > 5


def test_bench_rccl_one_rank():
    """bench.py under torch.distributed.run over RCCL (the driver's 1..8-GPU
    scaling command) with one rank: barrier, max-over-ranks all_reduce on a
    device tensor, one JSON line."""
    import json
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, NT_BENCH_BACKEND="nccl", NT_DIST_FORCE="1", HSA_ENABLE_IPC_MODE_LEGACY="0")
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK"):
        env.pop(k, None)
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "1",
           "--master-addr", "127.0.0.1", "--master-port", str(_port()), os.path.join(root, "bench.py"),
           "--gpus", "1", "--steps", "3", "--warmup", "1", "--config", "c10k", "--reads", "20000",
           "--no-cpu-baseline"]
    r = subprocess.run(cmd, env=env, check=True, timeout=240, capture_output=True, text=True)
    lines = [x for x in r.stdout.splitlines() if x.startswith("{")]
    assert len(lines) == 1, r.stdout
    d = json.loads(lines[0])
    assert d["n_gpus"] == 1 and d["value"] > 0


def test_bench_times_only_the_specialised_calling_kernel():
    """bench.py waits for the specialised calling kernel's build before its
    warm-up, so that no timed step runs the ahead-of-time kernel (VERDICT r3
    item 5): a batch of >= 65,536 reads reports only specialised calling
    launches, the calling kernel's own per-launch time and the exposed part."""
    import json
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0")
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "NT_CALL_JIT"):
        env.pop(k, None)
    r = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--steps", "3", "--warmup", "1",
                        "--config", "c10k", "--reads", "100000", "--no-cpu-baseline"],
                       env=env, check=True, timeout=240, capture_output=True, text=True)
    d = json.loads([x for x in r.stdout.splitlines() if x.startswith("{")][-1])
    rf = d["roofline"]
    assert rf["call_launches_timed"]["ahead_of_time"] == 0
    assert rf["call_launches_timed"]["specialised"] >= 3
    assert rf["call_kernel"].startswith("nt_call_jit")
    assert rf["call_kernel_avg_ms"] > 0 and rf["call_exposed_ms"] >= 0
