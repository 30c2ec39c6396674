"""--analysis post-processing of the summary rows (SURVEY §8(f) row 4;
NanoTel.R:2434-2508), host side.

    df_filtered = df_summary
      |> filter(telo_density_mismatch >= 0.75, Telomere_start_mismatch <= 134)
      |> arrange(desc(sequence_length))                        # stable
      |> mutate(TelLenMM_RunningMed = median(Telomere_length_mismatch[1:i]),
                SeqLen_minus_RunMed = sequence_length - TelLenMM_RunningMed)
      |> filter(SeqLen_minus_RunMed >= 134)

written as <barcode>_filtered_sorted_summary.csv (write_csv, the summary's
number formatting) and <barcode>_results.txt (n, median telomere length with
mismatch, % shorter than 2 kb).  NA comparisons drop the row, as dplyr's
filter does.  The ggplot2 figure (<barcode>_telomere_plot.png, NanoTel.R:
2486-2506) is drawn with matplotlib in ggplot2's layout with theme_prism's
look (12 x 6 in at 150 dpi, three lines over read_index, legend at the
bottom); it is not pixel-identical to R's (no ggplot2 rasteriser here).
"""
import heapq
import math
import os

from .io import format_double, r_as_character

# summary row fields (driver.chunk_rows): Serial, sequence_ID, sequence_length,
# then per pass: density, start, end, length
_LEN, _DMM, _SMM, _LMM = 2, 7, 8, 10
MIN_DENSITY_MM = 0.75  # NanoTel.R:2442
MAX_START_MM = 134     # NanoTel.R:2443, 2461


class _RunningMedian:
    """median(x[1:i]) for i = 1, 2, ... (R: the middle value for odd i, the
    mean of the two middle values for even i), two heaps."""

    def __init__(self):
        self.lo, self.hi = [], []  # max-heap (negated) / min-heap

    def push(self, x):
        if self.lo and x > -self.lo[0]:
            heapq.heappush(self.hi, x)
        else:
            heapq.heappush(self.lo, -x)
        if len(self.lo) > len(self.hi) + 1:
            heapq.heappush(self.hi, -heapq.heappop(self.lo))
        elif len(self.hi) > len(self.lo):
            heapq.heappush(self.lo, -heapq.heappop(self.hi))

    def median(self):
        if len(self.lo) > len(self.hi):
            return -self.lo[0]                 # odd: an element (integer in R)
        return (-self.lo[0] + self.hi[0]) / 2.0  # even: mean of the two, a double


def _keep_first(row):
    d, s = row[_DMM], row[_SMM]
    return d is not None and s is not None and d >= MIN_DENSITY_MM and s <= MAX_START_MM


def analyze(rows):
    """Returns (filtered rows with the two added columns, plot rows).  Plot
    rows = the sorted rows before the last filter as (read_index,
    sequence_length, Telomere_length_mismatch, TelLenMM_RunningMed)."""
    kept = [r for r in rows if _keep_first(r)]
    kept.sort(key=lambda r: -r[_LEN])  # arrange(desc()): stable, ties keep their order
    rm = _RunningMedian()
    out, plot = [], []
    for i, r in enumerate(kept, 1):
        rm.push(r[_LMM])
        med = rm.median()
        diff = r[_LEN] - med
        plot.append((i, r[_LEN], r[_LMM], med))
        if diff >= MAX_START_MM:
            out.append(list(r) + [med, diff])
    return out, plot


def median_text(values):
    """paste0() of median(): integer for an odd count, a double (R's
    as.character) for an even one, "NA" when empty."""
    v = sorted(values)
    n = len(v)
    if n == 0:
        return "NA"
    if n % 2:
        return str(int(v[n // 2]))
    return r_as_character((v[n // 2 - 1] + v[n // 2]) / 2.0)


def results_lines(barcode, filtered):
    n = len(filtered)
    lens = [r[_LMM] for r in filtered]
    pct = round(100 * sum(1 for x in lens if x < 2000) / n, 1) if n else float("nan")
    pct_s = "NaN" if math.isnan(pct) else r_as_character(pct)
    return [f"Results for {barcode}",
            "==========================================",
            f"Number of telomeric reads after filtration : {n}",
            f"Median telomere length with mismatch (bp)  : {median_text(lens)}",
            f"% of telomeres shorter than 2kb            : {pct_s}%"]


# scale_color_manual of NanoTel.R:2491-2495, in the legend's (alphabetical) order
PLOT_SERIES = (("Read Length", 1, "#E8735A"),
               ("Running Median Telomere Length", 3, "#4169E1"),
               ("Telomere Length (mismatch)", 2, "#228B22"))


def write_telomere_plot(path, plot):
    """<barcode>_telomere_plot.png: ggplot(df_for_plot, aes(x = read_index)) +
    three geom_line()s (NanoTel.R:2486-2506), title "Telomere Analysis", axis
    labels and the legend at the bottom as there; theme_prism's look: no grid,
    black axis lines with outward ticks, bold titles.  plot: analyze()'s plot
    rows.  An empty plot (no read kept) draws the empty panel, as ggplot2."""
    import matplotlib
    matplotlib.use("Agg")
    import matplotlib.pyplot as plt
    fig = plt.figure(figsize=(12, 6), dpi=150)
    try:
        ax = fig.add_subplot(1, 1, 1)
        x = [r[0] for r in plot]
        # ggplot2 geom_line: linewidth 0.5 mm = 1.42 pt; draw order = the layers
        for name, col, colour in (PLOT_SERIES[0], PLOT_SERIES[2], PLOT_SERIES[1]):
            ax.plot(x, [r[col] for r in plot], color=colour, linewidth=1.42, label=name)
        ax.set_title("Telomere Analysis", fontsize=14, fontweight="bold")
        ax.set_xlabel("Read (sorted by length, longest to shortest)", fontsize=14, fontweight="bold")
        ax.set_ylabel("Length (bp)", fontsize=14, fontweight="bold")
        for side in ("top", "right"):
            ax.spines[side].set_visible(False)
        for side in ("left", "bottom"):
            ax.spines[side].set_linewidth(1.0)
        ax.tick_params(direction="out", length=5, width=1.0, labelsize=12)
        ax.grid(False)
        handles, labels = ax.get_legend_handles_labels()
        order = [labels.index(n) for n, _, _ in PLOT_SERIES if n in labels]
        if order:
            ax.legend([handles[i] for i in order], [labels[i] for i in order], loc="upper center",
                      bbox_to_anchor=(0.5, -0.14), ncol=3, frameon=False, fontsize=12)
        fig.tight_layout()
        fig.savefig(path, dpi=150, format="png")
    finally:
        plt.close(fig)


def write_analysis(save_path, barcode, rows, columns, format_row, sci_threshold=None, plot_png=True):
    """Writes <barcode>_filtered_sorted_summary.csv, <barcode>_results.txt and
    (plot_png) <barcode>_telomere_plot.png; returns the plot rows."""
    filtered, plot = analyze(rows)
    with open(os.path.join(save_path, f"{barcode}_filtered_sorted_summary.csv"), "w", newline="") as f:
        f.write(",".join(list(columns) + ["TelLenMM_RunningMed", "SeqLen_minus_RunMed"]) + "\n")
        for r in filtered:
            f.write(format_row(r[:-2], sci_threshold) + "," + format_double(float(r[-2])) + ","
                    + format_double(float(r[-1])) + "\n")
    with open(os.path.join(save_path, f"{barcode}_results.txt"), "w") as f:
        for line in results_lines(barcode, filtered):
            f.write(line + "\n")
    if plot_png:
        write_telomere_plot(os.path.join(save_path, f"{barcode}_telomere_plot.png"), plot)
    return plot
