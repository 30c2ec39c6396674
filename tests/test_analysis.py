"""--analysis post-processing (NanoTel.R:2434-2508) on CPU: filter, stable
descending sort, running median of the mismatch telomere length, the second
filter, the CSV and the results text.  Checked against a direct restatement
of the dplyr pipeline (statistics.median over every prefix) and by hand."""
import os
import random
import statistics

from nanotel_amd import analysis, driver


def row(serial, n, dmm, smm, lmm, name=None):
    """A two-pass summary row; pass 1 copies pass 2 (only pass 2 is used)."""
    if smm is None:
        p = [None] * 4
    else:
        p = [dmm, smm, smm + lmm - 1, lmm]
    return [float(serial), name or f"r{serial}", n] + p + p


def direct(rows):
    kept = [r for r in rows if r[7] is not None and r[8] is not None and r[7] >= 0.75 and r[8] <= 134]
    kept = sorted(kept, key=lambda r: -r[2])
    out = []
    for i, r in enumerate(kept, 1):
        med = statistics.median([x[10] for x in kept[:i]])
        if r[2] - med >= 134:
            out.append(list(r) + [med, r[2] - med])
    return out


def test_running_median_and_filters_by_hand():
    rows = [row(1, 10000, 0.9, 1, 3000), row(2, 20000, 0.8, 50, 5000), row(3, 20000, 0.74, 1, 100),
            row(4, 20000, 0.99, 135, 100), row(5, 8000, 0.75, 134, 7000), row(6, 5100, 0.95, 1, 5000),
            row(7, 30000, 0.9, None, None), row(8, 20000, 0.76, 2, 4000)]
    out, plot = analysis.analyze(rows)
    # kept: 1, 2, 5, 6, 8; sorted by length desc, ties in input order: 2, 8, 1, 5, 6
    assert [p[0] for p in plot] == [1, 2, 3, 4, 5]
    assert [p[1] for p in plot] == [20000, 20000, 10000, 8000, 5100]
    # running medians: 5000; 4500.0; 4000; 4500.0; 5000
    assert [p[3] for p in plot] == [5000, 4500.0, 4000, 4500.0, 5000]
    # diffs: 15000, 15500, 6000, 3500, 100 (< 134: dropped)
    assert [int(r[0]) for r in out] == [2, 8, 1, 5]
    assert out == direct(rows)


def test_matches_direct_restatement_random():
    rng = random.Random(5)
    rows = []
    for i in range(600):
        n = rng.choice([rng.randint(1000, 60000), 20000])  # ties in sequence_length
        if rng.random() < 0.1:
            rows.append(row(i + 1, n, None, None, None))
            continue
        lmm = rng.randint(30, n)
        rows.append(row(i + 1, n, rng.choice([0.74, 0.75, 0.8, rng.random()]), rng.choice([1, 134, 135, 500]), lmm))
    out, _ = analysis.analyze(rows)
    ref = direct(rows)
    assert len(out) == len(ref) > 10
    for a, b in zip(out, ref):
        assert a[:-2] == b[:-2] and float(a[-2]) == float(b[-2]) and float(a[-1]) == float(b[-1])


def test_written_files(tmp_path):
    rows = [row(1, 10000, 0.9, 1, 3000), row(2, 20000, 0.8, 50, 1500), row(3, 15000, 0.97, 3, 2500)]
    analysis.write_analysis(str(tmp_path), "bc", rows, driver.columns(False), driver.format_row)
    csv = (tmp_path / "bc_filtered_sorted_summary.csv").read_text().splitlines()
    assert csv[0] == ",".join(driver.BASE_COLUMNS) + ",TelLenMM_RunningMed,SeqLen_minus_RunMed"
    # sorted 2 (1500), 3 (2500 -> median 2000.0), 1 (3000 -> median 2500)
    assert csv[1] == "2,r2,20000,0.8,50,1549,1500,0.8,50,1549,1500,1500,18500"
    assert csv[2] == "3,r3,15000,0.97,3,2502,2500,0.97,3,2502,2500,2000,13000"
    assert csv[3] == "1,r1,10000,0.9,1,3000,3000,0.9,1,3000,3000,2500,7500"
    txt = (tmp_path / "bc_results.txt").read_text().splitlines()
    assert txt == ["Results for bc", "==========================================",
                   "Number of telomeric reads after filtration : 3",
                   "Median telomere length with mismatch (bp)  : 2500",
                   "% of telomeres shorter than 2kb            : 33.3%"]


def test_example_summary_filters_to_nothing(tmp_path):
    """Example/Example_output: only read 1 passes the first filter and its
    length minus the running median is 0 (< 134): header only, NA / NaN."""
    here = os.path.dirname(os.path.abspath(__file__))
    lines = open(os.path.join(here, "golden", "example_summary.csv")).read().splitlines()[1:]
    rows = []
    for ln in lines:
        f = ln.split(",")
        rows.append([float(f[0]), f[1], int(f[2]), float(f[3]), int(f[4]), int(f[5]), int(f[6]),
                     float(f[7]), int(f[8]), int(f[9]), int(f[10])])
    analysis.write_analysis(str(tmp_path), "sample.fasta", rows, driver.columns(False), driver.format_row)
    assert len((tmp_path / "sample.fasta_filtered_sorted_summary.csv").read_text().splitlines()) == 1
    txt = (tmp_path / "sample.fasta_results.txt").read_text().splitlines()
    assert txt[2:] == ["Number of telomeric reads after filtration : 0",
                       "Median telomere length with mismatch (bp)  : NA",
                       "% of telomeres shorter than 2kb            : NaN%"]


def test_median_text_types():
    assert analysis.median_text([3, 1, 2]) == "2"
    assert analysis.median_text([1, 2]) == "1.5"
    assert analysis.median_text([100000, 100000]) == "1e+05"  # a double: as.character
    assert analysis.median_text([100000]) == "100000"           # an integer
    assert analysis.median_text([]) == "NA"


def test_telomere_plot_png(tmp_path):
    """<barcode>_telomere_plot.png (NanoTel.R:2486-2506): 12 x 6 in at 150 dpi,
    the three series in their scale_color_manual colours.  Not pixel-identical
    to ggplot2 (parity unpinned: no R here)."""
    from PIL import Image
    rows = [row(i, 20000 - 37 * i, 0.9, 1, 1000 + 13 * (i % 50)) for i in range(1, 200)]
    plot = analysis.write_analysis(str(tmp_path), "bc", rows, driver.columns(False), driver.format_row)
    assert len(plot) == 199 and [p[0] for p in plot] == list(range(1, 200))
    im = Image.open(tmp_path / "bc_telomere_plot.png").convert("RGB")
    assert im.size == (1800, 900)
    colours = {c for _, c in im.getcolors(1 << 20)}
    for _, _, hexc in analysis.PLOT_SERIES:
        rgb = tuple(int(hexc[i:i + 2], 16) for i in (1, 3, 5))
        assert rgb in colours, hexc
    # no rows kept: the empty panel is still written
    analysis.write_analysis(str(tmp_path), "empty", [], driver.columns(False), driver.format_row)
    assert Image.open(tmp_path / "empty_telomere_plot.png").size == (1800, 900)
