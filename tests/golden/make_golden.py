"""Regenerate the committed golden fixtures from the reference's Example/ data.

Run in the build container (where /root/reference exists):
    python tests/golden/make_golden.py

Outputs (all *data*, no reference source):
  sample.fasta                    -- Example/sample.fasta (the C1 input, 4 reads)
  example_summary.csv             -- Example/Example_output/summary.csv (2023 code version)
  reads/{1..4}.fasta              -- Example/Example_output/reads/*.fasta (written telomeric reads)
  eps/read{1..4}.eps              -- Example/Example_output/single_read_plots_adj/read*.eps (plots)
  jpeg_adj/read{1..4}.jpeg        -- Example/Example_output/single_read_plots_adj/read*.jpeg (R's
                                     cairo jpeg() of the same plots; pixel parity, tests/test_plots.py)
  example_window_counts.json      -- per-window covered-base counts for P1 (exact)
                                     and P2 (1 mismatch), decoded from the density
                                     polygons of Example_output/single_read_plots_adj/read*.eps

EPS decoding (R's postscript device, devPS.c PS_Polygon): the polygon for a
pass is drawn from (1, 0) through (start_i, density_i) for every window, then
(n, d_last), (n, 0).  Coordinates are printed with 2 decimals; every 100th
point is an absolute "x y lineto", the rest "dx dy l" with dx/dy the
difference of the 2-decimal-rounded absolute coordinates.  y = 87.20 + 344*d
(ylim c(0,1) on a 371.52-pt region with 4% extension).  The first polygon
(/bg orange) is the mismatch pass (subs_mismatch), the second (/bg salmon) the
exact pass (NanoTel.R:1329-1337).  density_i*width_i is an integer count;
|error| <= 0.005*150/344 < 0.003, so counts are recovered exactly.
"""
import json
import os
import shutil
import sys

REF = "/root/reference/Example"
HERE = os.path.dirname(os.path.abspath(__file__))


def read_fasta(path):
    names, seqs, cur = [], [], []
    with open(path) as f:
        for line in f:
            line = line.rstrip("\r\n")
            if line.startswith(">"):
                if names:
                    seqs.append("".join(cur))
                names.append(line[1:])
                cur = []
            else:
                cur.append(line.strip())
    seqs.append("".join(cur))
    return names, seqs


def polygons(eps_text):
    """Return {color_tag: [y in hundredths, ...]} for the two density polygons."""
    lines = eps_text.splitlines()
    out = {}
    i = 0
    tag = None
    while i < len(lines):
        ln = lines[i].strip()
        if ln.startswith("/bg {"):
            tag = ln
        if ln == "np" and tag is not None and ("0.6471" in tag or "0.9804" in tag):
            x0, y0, _ = lines[i + 1].split()
            X = [round(float(x0) * 100)]
            Y = [round(float(y0) * 100)]
            j = i + 2
            while not lines[j].startswith("cp"):
                parts = lines[j].split()
                if parts[-1] == "lineto":
                    X.append(round(float(parts[0]) * 100))
                    Y.append(round(float(parts[1]) * 100))
                else:
                    assert parts[-1] == "l", parts
                    X.append(X[-1] + round(float(parts[0]) * 100))
                    Y.append(Y[-1] + round(float(parts[1]) * 100))
                j += 1
            out["p2" if "0.6471" in tag else "p1"] = (X, Y)
            i = j
        i += 1
    return out


def main():
    os.makedirs(HERE, exist_ok=True)
    shutil.copyfile(os.path.join(REF, "sample.fasta"), os.path.join(HERE, "sample.fasta"))
    shutil.copyfile(os.path.join(REF, "Example_output", "summary.csv"),
                    os.path.join(HERE, "example_summary.csv"))
    # the telomeric reads as the reference wrote them (reads/<serial>.fasta, 2023 version)
    os.makedirs(os.path.join(HERE, "reads"), exist_ok=True)
    for serial in range(1, 5):
        shutil.copyfile(os.path.join(REF, "Example_output", "reads", f"{serial}.fasta"),
                        os.path.join(HERE, "reads", f"{serial}.fasta"))
    # the single-read EPS plots as the reference wrote them (expected outputs of plots.py)
    os.makedirs(os.path.join(HERE, "jpeg_adj"), exist_ok=True)
    for serial in range(1, 5):
        shutil.copyfile(os.path.join(REF, "Example_output", "single_read_plots_adj", f"read{serial}.jpeg"),
                        os.path.join(HERE, "jpeg_adj", f"read{serial}.jpeg"))
    os.makedirs(os.path.join(HERE, "eps"), exist_ok=True)
    for serial in range(1, 5):
        shutil.copyfile(os.path.join(REF, "Example_output", "single_read_plots_adj", f"read{serial}.eps"),
                        os.path.join(HERE, "eps", f"read{serial}.eps"))
    names, seqs = read_fasta(os.path.join(REF, "sample.fasta"))
    L = 100
    result = {"L": L, "min_density": 0.6, "patterns": "TTAGGG", "reads": []}
    for serial, (name, seq) in enumerate(zip(names, seqs), start=1):
        n = len(seq)
        # split_telo window widths (NanoTel.R:199-227)
        starts = list(range(1, n + 1, L))
        ends = [s + L - 1 for s in starts]
        ends[-1] = n
        if n - starts[-1] < L / 2:
            starts, ends = starts[:-1], ends[:-1]
            ends[-1] = n
        widths = [e - s + 1 for s, e in zip(starts, ends)]
        with open(os.path.join(REF, "Example_output", "single_read_plots_adj",
                               f"read{serial}.eps")) as f:
            polys = polygons(f.read())
        rec = {"serial": serial, "name": name, "n": n, "n_windows": len(widths)}
        for key in ("p1", "p2"):
            X, Y = polys[key]
            m = len(widths)
            assert len(Y) == m + 3, (serial, key, len(Y), m)
            y0 = Y[0]
            counts = []
            for w, yy in zip(widths, Y[1:m + 1]):
                d = (yy - y0) / 100.0 / 344.0
                k = round(d * w)
                assert abs(d * w - k) < 0.01, (serial, key, d, w)
                counts.append(k)
            # polygon x coordinates are the window starts (device coords; monotone check)
            assert all(X[i + 1] >= X[i] for i in range(m)), (serial, key)
            rec[key + "_counts"] = counts
        rec["widths"] = widths
        result["reads"].append(rec)
    with open(os.path.join(HERE, "example_window_counts.json"), "w") as f:
        json.dump(result, f, indent=1)
    total = sum(2 * r["n_windows"] for r in result["reads"])
    print("windows decoded:", total)


if __name__ == "__main__":
    sys.exit(main())
