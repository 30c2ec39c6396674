"""One line per bench.py log: value, step, scan launch, launches, frac, exposed calling."""
import json
import sys

for f in sys.argv[1:]:
    try:
        d = json.loads(open(f).read().strip().splitlines()[-1])
        r = d["roofline"]
        print(f, d["value"], d["ms_per_step"], r["kernel_avg_ms"], r["kernel_launches_per_step"], r["frac"],
              "call exposed", r["call_exposed_ms"], d["config"].get("env_knobs"))
    except Exception as e:  # noqa: BLE001 (a missing or partial log)
        print(f, "no bench line:", type(e).__name__)
