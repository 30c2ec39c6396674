"""Sharded serial assignment: per-rank chunks + one
all_reduce(MAX) of the chunks' relative maxima must reproduce the reference's
sequential serial recurrence (A15, NanoTel.R:2050-2070, 2234-2258) exactly,
including the -Inf serial_start while no row exists.  CPU only (gloo)."""
import os
import socket
import tempfile

import numpy as np
import pytest

import _oracle as O
from nanotel_amd import shard


def _oracle_sequential(flags_per_chunk):
    """The reference recurrence chunk by chunk (CPU oracle, nto_assign_serials)."""
    ss, mx = 1.0, float("-inf")
    out = []
    for f in flags_per_chunk:
        ser, order, ss, mx = O.assign_serials(list(f), ss, mx)
        out.append((np.array(ser, np.float64), order))
    return out


def _chunks(seed, n_chunks=23):
    rng = np.random.default_rng(seed)
    out = []
    for k in range(n_chunks):
        n = int(rng.choice([0, 1, 5, 7, 8, 9, 33, 250]))
        p = [0.0, 0.1, 0.5, 1.0][k % 4]
        out.append((rng.random(n) < p).astype(np.uint8))
    return out


def _same(a, b):
    a, b = np.asarray(a, np.float64), np.asarray(b, np.float64)
    return a.shape == b.shape and bool(np.all((a == b) | (np.isnan(a) & np.isnan(b))))


@pytest.mark.parametrize("seed", [1, 2, 3])
def test_recurrence_matches_sequential(seed):
    flags = _chunks(seed)
    ref = _oracle_sequential(flags)
    rels = [shard.chunk_relative(f) for f in flags]
    starts = shard.serial_starts([r[2] for r in rels])
    for k, (rel, order, _) in enumerate(rels):
        assert _same(shard.assign_chunk_serials(rel, starts[k]), ref[k][0]), k
        assert list(order) == list(ref[k][1]), k
    # the library's own sequential driver agrees too
    for k, ser in enumerate(shard.sequential_serials(flags)):
        assert _same(ser, ref[k][0])


def test_leading_empty_chunks_give_minus_inf():
    # max(numeric(0)) + 1 = -Inf: once the first chunk has no row, every later
    # serial_start is -Inf (reference behaviour, NanoTel.R:2258)
    flags = [np.zeros(10, np.uint8), np.ones(3, np.uint8), np.ones(9, np.uint8)]
    ref = [r[0] for r in _oracle_sequential(flags)]
    assert np.all(np.isneginf(ref[1])) and np.all(np.isneginf(ref[2]))
    rels = [shard.chunk_relative(f) for f in flags]
    starts = shard.serial_starts([r[2] for r in rels])
    assert starts[0] == 1.0 and np.isneginf(starts[1]) and np.isneginf(starts[2])


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _rank_main(rank, world, port, seed, out_path):
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    flags = _chunks(seed)  # every rank knows the chunk layout, scans only its own chunks
    mine = shard.local_chunks(len(flags), rank, world)
    rel = {k: shard.chunk_relative(flags[k]) for k in mine}
    all_max, failed = shard.exchange_rel_max({k: rel[k][2] for k in mine}, len(flags))
    assert not failed
    starts = shard.serial_starts(all_max)
    rows = {}
    for k in mine:
        ser = shard.assign_chunk_serials(rel[k][0], starts[k])
        rows[k] = [(k, int(j), float(ser[j])) for j in rel[k][1]]  # group-major row order
    merged = shard.gather_rows(rows)
    if rank == 0:
        np.save(out_path, np.array(merged, dtype=np.float64).reshape(-1, 3))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_gloo_sharded_serials_match_sequential(world):
    import torch.multiprocessing as mp
    seed = 11
    with tempfile.TemporaryDirectory() as d:
        out = os.path.join(d, "rows.npy")
        mp.spawn(_rank_main, args=(world, _free_port(), seed, out), nprocs=world, join=True)
        got = np.load(out)
    flags = _chunks(seed)
    exp = []
    for k, (ser, order) in enumerate(_oracle_sequential(flags)):
        exp += [(k, int(j), float(ser[j])) for j in order]
    exp = np.array(exp, dtype=np.float64).reshape(-1, 3)
    assert got.shape == exp.shape
    assert _same(got, exp)
