"""bench.py's launch contract without a GPU: --gpus N must match the ranks
launched (the driver computes scaling from the per-N values)."""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_bench_rank_count_mismatch_fails():
    """Launched with fewer ranks than --gpus, bench.py exits non-zero (it never
    reports a 1-GPU number as an N-GPU one)."""
    import subprocess
    import sys
    root = ROOT
    env = dict(os.environ, WORLD_SIZE="1", RANK="0", LOCAL_RANK="0", HSA_ENABLE_IPC_MODE_LEGACY="0")
    r = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--gpus", "2", "--steps", "1",
                        "--warmup", "0", "--config", "c10k", "--reads", "1000", "--no-cpu-baseline"],
                       env=env, timeout=120, capture_output=True, text=True)
    assert r.returncode != 0 and "WORLD_SIZE" in r.stderr


def test_bench_rejects_zero_gpus():
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "0"], timeout=60,
                       capture_output=True, text=True)
    assert r.returncode != 0
