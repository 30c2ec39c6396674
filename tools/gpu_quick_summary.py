"""Summary of tools/gpu_quick.sh's outputs for a tag."""
import json, sys
tag = sys.argv[1] if len(sys.argv) > 1 else "q"
for f, pick in (("t", lambda l: "passed" in l or "failed" in l),):
    try:
        for l in open(f"gpurun_out/{f}_{tag}.log"):
            if pick(l):
                print(l.rstrip())
    except OSError:
        print(f"no {f}_{tag}.log")
try:
    d = json.loads(open(f"gpurun_out/b_{tag}.log").read().strip().splitlines()[-1])
    r = d["roofline"]
    print("value", d["value"], "ms/step", d["ms_per_step"], "scan ms", r["kernel_avg_ms"], "frac", r["frac"],
          "call exposed", r["call_exposed_ms"])
except Exception as e:
    print("no bench line", e)
