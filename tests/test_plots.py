"""Single-read plots (plots.py; NanoTel.R:1271-1624, 1876-1912) on CPU.

* The reference's Example plots (single_read_plots_adj/read1-4.eps, committed
  as tests/golden/eps) are reproduced byte for byte from the golden window
  counts and summary rows (tests/golden/make_golden.py);
* every branch of the two plot functions (no exact telomere, no mismatch
  telomere, TVR pass found or not) writes a well-formed EPS and JPEGs;
* x-axis label thinning keeps labels at least one "m" apart.
"""
import json
import os
import re

import pytest

from nanotel_amd import plots

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def _golden():
    g = json.load(open(os.path.join(GOLD, "example_window_counts.json")))
    rows = [ln.split(",") for ln in open(os.path.join(GOLD, "example_summary.csv")).read().splitlines()[1:]]
    return g, rows


@pytest.mark.parametrize("serial", [1, 2, 3, 4])
def test_example_eps_byte_identical(serial):
    g, rows = _golden()
    rec, row = g["reads"][serial - 1], rows[serial - 1]
    subs = plots.window_table(rec["n"], g["L"], rec["p1_counts"])
    subs_mm = plots.window_table(rec["n"], g["L"], rec["p2_counts"])
    ops = plots.plot_ops(rec["n"], rec["n"], subs, subs_mm, int(row[4]), int(row[5]), int(row[8]), int(row[9]))
    assert plots.render_eps(ops) == open(os.path.join(GOLD, "eps", f"read{serial}.eps")).read()


def _polys(eps):
    return re.findall(r"/bg \{ ([^}]*) \} def\n(?:[^\n]*\n)*?np\n ", eps)


CASES = [
    # seq_start, seq_end, gray_start, gray_end, tvr (start, end) or None
    (1, 3000, 1, 3400, None),
    (200, 3000, 150, 3400, None),
    (-1, -1, 400, 2000, None),
    (1, 3000, -1, -1, None),
    (1, 3000, 1, 3400, (1, 3600)),
    (300, 3000, 250, 3400, (100, 3600)),
    (1, 3000, -1, -1, (-1, -1)),
    (1, 3000, -1, -1, (1, 3500)),
    (-1, -1, 400, 2000, (300, 2500)),
    (-1, -1, 400, 2000, (-1, -1)),
]


@pytest.mark.parametrize("case", CASES)
def test_branches_write_files(tmp_path, case):
    s1, e1, s2, e2, tvr = case
    n, L = 7345, 100
    nw = 73
    c1 = [min(100, (k * 7) % 101) for k in range(nw)]
    c2 = [min(100, c + 3) for c in c1]
    c3 = [min(100, c + 5) for c in c1]
    for d in ("single_read_plots", "single_read_plots_adj"):
        os.makedirs(tmp_path / d)
    kw = {}
    if tvr is not None:
        kw = dict(subs_tvr=plots.window_table(n, L, c3), tvr_start=tvr[0], tvr_end=tvr[1])
    plots.write_read_plots(str(tmp_path), "12", n, plots.window_table(n, L, c1), plots.window_table(n, L, c2),
                           s1, e1, s2, e2, **kw)
    eps = (tmp_path / "single_read_plots_adj" / "read12.eps").read_text()
    assert eps.startswith("%!PS-Adobe-3.0 EPSF-3.0") and eps.endswith("%%EOF\n")
    assert eps.count("cp p3") == (3 if tvr is not None else 2) and eps.count("cp p1") == 1
    legend = 7 if tvr is not None else 5
    assert eps.count("findfont 14 s") == 2  # legend, main title
    assert len(re.findall(r"\) 0 0 t\n|\) 0 ta\n", eps.split("/Font1 findfont 14 s")[1].split("cl\n")[0])) == legend
    assert "(Read length: 7345 " in eps
    from PIL import Image
    for d in ("single_read_plots", "single_read_plots_adj"):
        im = Image.open(tmp_path / d / "read12.jpeg")
        assert im.size == (750, 300)


def test_axis_label_thinning():
    fig_ops = plots.plot_ops(plots.MAX_LENGTH, 50000, ([1], [0.5]), ([1], [0.5]), 1, 100, 1, 120)
    labs = [op for op in fig_ops if op[0] == "text" and op[3].endswith("kb")]
    assert labs[0][3] == "0.0kb" and 3 < len(labs) < 100
    gap = plots.str_width("m", 1, 12)
    for a, b in zip(labs, labs[1:]):
        wa, wb = plots.str_width(a[3], 1, 12), plots.str_width(b[3], 1, 12)
        assert (b[1] - 0.5 * wb) - (a[1] + 0.5 * wa) >= gap - 1e-9


def test_plot_worker_processes(tmp_path):
    """The driver's spawned plot workers (large chunks) write the same files
    as the in-process writer."""
    from nanotel_amd import driver
    for d in ("single_read_plots", "single_read_plots_adj"):
        os.makedirs(tmp_path / "a" / d)
        os.makedirs(tmp_path / "b" / d)
    g, rows = _golden()
    jobs = []
    for rec, row in zip(g["reads"], rows):
        t1 = plots.window_table(rec["n"], g["L"], rec["p1_counts"])
        t2 = plots.window_table(rec["n"], g["L"], rec["p2_counts"])
        jobs.append((str(rec["serial"]), rec["n"], t1, t2, int(row[4]), int(row[5]), int(row[8]), int(row[9])))
    pool = driver._plot_pool()
    try:
        futs = [pool.submit(plots.write_read_plots, str(tmp_path / "a"), *j) for j in jobs]
        for f in futs:
            f.result()
    finally:
        pool.shutdown()
    for j in jobs:
        plots.write_read_plots(str(tmp_path / "b"), *j)
    for j in jobs:
        for rel in (f"single_read_plots_adj/read{j[0]}.eps", f"single_read_plots/read{j[0]}.jpeg"):
            assert (tmp_path / "a" / rel).read_bytes() == (tmp_path / "b" / rel).read_bytes()
        assert (tmp_path / "a" / f"single_read_plots_adj/read{j[0]}.eps").read_text() == open(
            os.path.join(GOLD, "eps", f"read{j[0]}.eps")).read()


def _psnr(a, b):
    import numpy as np
    mse = float(((a - b) ** 2).mean())
    return 10 * np.log10(255.0 ** 2 / max(mse, 1e-9))


@pytest.mark.parametrize("serial", [1, 2, 3, 4])
def test_example_jpeg_pixels_match_reference(tmp_path, serial):
    """The Example's single_read_plots_adj/read<serial>.jpeg (R's cairo jpeg()
    device, NanoTel.R:1876-1896) against ours, drawn from the golden window
    counts: anti-aliased at R's 72 dpi, lines of 0.75 px, text set to the
    Helvetica widths (DejaVu glyphs: the only face here).  Thresholds:
      * the plot region (the density polygons, the telomere bars, axes' box,
        no text): PSNR >= 28 dB, mean absolute difference <= 3 (of 255);
      * the whole image (glyph shapes differ: DejaVu against R's Helvetica
        substitute): PSNR >= 18.5 dB, mean absolute difference <= 8.
    (The reference's full-axis single_read_plots/read*.jpeg come from an older
    plot -- no gray area in the legend, "read length" in lower case -- like its
    summary.csv, so only the _adj plots are compared.)"""
    import numpy as np
    from PIL import Image
    g, rows = _golden()
    rec, row = g["reads"][serial - 1], rows[serial - 1]
    subs = plots.window_table(rec["n"], g["L"], rec["p1_counts"])
    subs_mm = plots.window_table(rec["n"], g["L"], rec["p2_counts"])
    for d in ("single_read_plots", "single_read_plots_adj"):  # create_dirs (NanoTel.R:1978-1996)
        (tmp_path / d).mkdir()
    plots.write_read_plots(str(tmp_path), str(serial), rec["n"], subs, subs_mm, int(row[4]), int(row[5]),
                           int(row[8]), int(row[9]))
    a = np.asarray(Image.open(tmp_path / "single_read_plots_adj" / f"read{serial}.jpeg").convert("RGB")).astype(float)
    b = np.asarray(Image.open(os.path.join(GOLD, "jpeg_adj", f"read{serial}.jpeg")).convert("RGB")).astype(float)
    assert a.shape == b.shape == (300, 750, 3)
    r = (slice(60, 225), slice(62, 575))  # inside the plot box, left of the legend
    assert _psnr(a[r], b[r]) >= 28.0 and np.abs(a[r] - b[r]).mean() <= 3.0
    assert _psnr(a, b) >= 18.5 and np.abs(a - b).mean() <= 8.0
