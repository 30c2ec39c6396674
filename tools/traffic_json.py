"""profiles/pmc_traffic.json from tools/profile_round.sh output: per-launch
HBM bytes of the scan kernel (FETCH_SIZE x 1024 x 2 -- gfx950 reports half of
wide streaming reads, MI355X_MICROARCH.md "HBM" -- plus WRITE_SIZE x 1024).
usage: python tools/traffic_json.py OUTDIR CONFIG READS JIT(0/1) [dest]"""
import csv
import glob
import json
import os
import sys


def per_dispatch(path, counter, match):
    vals = []
    for f in glob.glob(os.path.join(path, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if r["Counter_Name"] == counter and match(r["Kernel_Name"]):
                vals.append(float(r["Counter_Value"]))
    return vals


def main():
    out, config, reads, jit = sys.argv[1], sys.argv[2], int(sys.argv[3]), bool(int(sys.argv[4]))
    dest = sys.argv[5] if len(sys.argv) > 5 else "profiles/pmc_traffic.json"
    is_scan = lambda k: "nt_scan" in k or "nt_tscan" in k  # noqa: E731 (per-read or bundle scan)
    is_call = lambda k: "nt_call_kernel" in k or "nt_call_jit" in k  # noqa: E731 (AOT or specialised)
    res = {"config": config, "reads": reads, "jit": jit,
           "method": "rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE (separate passes), per dispatch mean; "
                     "read bytes = FETCH_SIZE*1024*2 (gfx950 halves wide streaming reads), "
                     "write bytes = WRITE_SIZE*1024"}
    for name, m in (("scan", is_scan), ("call", is_call)):
        f = per_dispatch(os.path.join(out, "FETCH_SIZE"), "FETCH_SIZE", m)
        w = per_dispatch(os.path.join(out, "WRITE_SIZE"), "WRITE_SIZE", m)
        if not f or not w:
            raise SystemExit(f"no {name} dispatches found")
        rd = sum(f) / len(f) * 1024 * 2
        wr = sum(w) / len(w) * 1024
        res[f"{name}_read_bytes_per_launch"] = rd
        res[f"{name}_write_bytes_per_launch"] = wr
    res["hbm_bytes_per_launch"] = res["scan_read_bytes_per_launch"] + res["scan_write_bytes_per_launch"]
    json.dump(res, open(dest, "w"), indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
