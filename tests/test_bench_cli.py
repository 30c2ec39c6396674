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


def test_bench_refuses_debug_environment():
    """Timing builds and skipped kernels change what a step computes: bench.py
    exits non-zero before touching the GPU when any such variable is set
    (VERDICT r4 item 6), and records the other NT_* knobs in its line."""
    sys.path.insert(0, ROOT)
    import bench
    for var, val in (("NT_DBG_SKIP_CALL", "1"), ("NT_JIT_OPTS", "-DNT_TS_DBG_NOWALK=1"), ("NT_TSCAN", "0"),
                     ("NT_HOST_TLAYOUT", "1"), ("NT_TS_DBG_NOOUT", "1")):
        env = dict(os.environ, **{var: val})
        assert bench.refused_env(env) == [f"{var}={val}"]
        r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--steps", "1", "--warmup", "0"],
                           env=env, timeout=60, capture_output=True, text=True)
        assert r.returncode == 2 and var in r.stderr, (var, r.returncode, r.stderr[-400:])
    clean = {k: v for k, v in os.environ.items() if not k.startswith("NT_")}
    assert bench.refused_env(clean) == []
    assert bench.env_knobs(dict(clean, NT_TSUB="2", NT_JIT_CACHE="/x")) == {"NT_JIT_CACHE": "/x", "NT_TSUB": "2"}


def test_bench_default_is_the_metric_configuration():
    """The driver runs bench.py without --config: its default is BASELINE.json
    configs[4]'s per-GPU shard (12.5 M x 50 kb, TTAGGG), the configuration the
    headline metric is quoted on."""
    import json
    sys.path.insert(0, ROOT)
    import bench
    src = open(os.path.join(ROOT, "bench.py")).read()
    assert 'ap.add_argument("--config", default="c5"' in src
    cfg = bench.CONFIGS["c5"]
    assert (cfg["reads"], cfg["read_len"], cfg["patterns"], cfg["tvr"]) == (12_500_000, 50_000, "TTAGGG", None)
    base = json.load(open(os.path.join(ROOT, "BASELINE.json")))
    assert "TTAGGG, 50 kb reads" in base["metric"] and bench.METRICS["c5"].startswith("Gbases/s scanned (TTAGGG, 50 kb")
    assert "100M" in base["configs"][4] and 100_000_000 // 8 == cfg["reads"]
