"""<save_path>/log/run.log in the layout logr 1.3.4 gives NanoTel's log
(NanoTel.R:2347-2427, 2510-2516; pinned by Example/Example_output/log/run.log).

* log_open(<save_path>/run.log): logr puts the file in a log/ directory
  beside it and writes a header block -- a rule of 73 '=', Log Path, Working
  Directory, User Name, R Version, Machine, Operating System, Base / Other
  Packages, Log Start Time, the rule again, a blank line.  The R-specific
  entries name this build instead (there is no R here);
* log_print(<string>): the text, a space, a line break and a blank line;
* log_print(summary(x)): R's print of a summaryDefault (4 significant digits,
  common decimals, names and values right-aligned in columns of one width,
  an "NA's" column when x has NAs), then a blank line;
* log_close(footer = FALSE) (NanoTel.R:2514): no footer.
"""
import getpass
import math
import os
import platform
import time

import numpy as np

RULE = "=" * 73 + " "


def r_time(t=None):
    """toString(Sys.time()) with the microseconds (as in Example run.log)."""
    t = time.time() if t is None else t
    return time.strftime("%Y-%m-%d %H:%M:%S", time.localtime(t)) + ".%06d" % int(round((t % 1) * 1e6) % 1000000)


def _sig_info(x, digits):
    """R's scientific(): (kpower, nsig) of |x| rounded to `digits` significant digits."""
    if x == 0:
        return 0, 1
    a = abs(x)
    kp = int(math.floor(math.log10(a)))
    m = round(a / 10.0 ** kp * 10 ** (digits - 1))
    if m >= 10 ** digits:
        kp += 1
        m = round(a / 10.0 ** kp * 10 ** (digits - 1))
    nsig = digits
    while nsig > 1 and m % 10 == 0:
        m //= 10
        nsig -= 1
    return kp, nsig


def r_format(values, digits=4):
    """format(x, digits = digits) of a numeric vector in fixed notation: the
    fewest decimals (common to all) that show every value to `digits`
    significant digits, right-aligned to a common width; NA / NaN / Inf as R."""
    rgt, fin = 0, []
    for x in values:
        if x is None or not math.isfinite(x):
            continue
        kp, nsig = _sig_info(x, digits)
        rgt = max(rgt, nsig - kp - 1)
        fin.append(x)
    rgt = min(max(rgt, 0), 15)
    out = []
    for x in values:
        if x is None:
            out.append("NA")
        elif math.isnan(x):
            out.append("NaN")
        elif math.isinf(x):
            out.append("Inf" if x > 0 else "-Inf")
        else:
            out.append("%.*f" % (rgt, x))
    w = max((len(s) for s in out), default=0)
    return [s.rjust(w) for s in out]


def _zapsmall(v, digits):
    """zapsmall(x, digits): round to digits significant of the largest |x|."""
    fin = [abs(x) for x in v if math.isfinite(x)]
    if not fin or max(fin) == 0:
        return v
    d = max(0, digits - int(math.ceil(math.log10(max(fin)))))
    return [round(x, d) if math.isfinite(x) else x for x in v]


class ValueCounts:
    """A numeric column kept as its distinct values and their counts (plus an
    NA count), merged chunk by chunk: summary() of a column of 10^8 reads
    without holding it.  Integral values (read and telomere lengths) make the
    mean exact: their sum is an exact integer below 2^53."""

    def __init__(self):
        self.vals = np.zeros(0, np.float64)
        self.cnts = np.zeros(0, np.int64)
        self.na = 0

    def add(self, x):
        """x: array (NaN = NA) or another ValueCounts."""
        if isinstance(x, ValueCounts):
            v, c, na = x.vals, x.cnts, x.na
        else:
            v = np.asarray(x, np.float64)
            nan = np.isnan(v)
            na = int(nan.sum())
            v, c = np.unique(v[~nan], return_counts=True)
        self.na += na
        if v.size:
            u, inv = np.unique(np.concatenate([self.vals, v]), return_inverse=True)
            self.cnts = np.bincount(inv, weights=np.concatenate([self.cnts, c]), minlength=u.size).astype(np.int64)
            self.vals = u
        return self

    @property
    def n(self):
        return int(self.cnts.sum())

    def order_stat(self, i):
        """The i-th smallest value (0-based) of the column without its NAs."""
        return float(self.vals[int(np.searchsorted(np.cumsum(self.cnts), i, side="right"))])

    def quantile(self, q):
        """np.quantile(column, q) (method 'linear' = R's type 7), same arithmetic."""
        n = self.n
        h = (n - 1) * q
        lo = math.floor(h)
        a, b = self.order_stat(lo), self.order_stat(min(lo + 1, n - 1))
        t = h - lo
        d = b - a
        return b - d * (1.0 - t) if t >= 0.5 else a + d * t

    def mean(self):
        """np.mean of the column: for integral values its pairwise float64 sum
        is the exact integer sum (below 2^53), as here"""
        if np.all(self.vals == np.round(self.vals)) and np.abs(self.vals).max(initial=0) < 2 ** 31:
            return float(int(np.dot(self.vals.astype(np.int64), self.cnts))) / self.n
        return float(np.dot(self.vals, self.cnts)) / self.n


def r_summary(x):
    """summary(x) of a numeric vector: (names, values, NA count) -- Min, the
    type-7 quartiles, median, mean, max; NA's when x holds NAs."""
    if isinstance(x, ValueCounts):
        names = ["Min.", "1st Qu.", "Median", "Mean", "3rd Qu.", "Max."]
        if x.n == 0:
            return names, [None, None, None, float("nan"), None, None], x.na
        q = [x.quantile(p) for p in (0, 0.25, 0.5, 0.75, 1.0)]
        return names, [q[0], q[1], q[2], x.mean(), q[3], q[4]], x.na
    if isinstance(x, np.ndarray):  # (NA as NaN): no per-element Python work for millions of reads
        v = x.astype(np.float64, copy=False)
    else:
        v = np.asarray([np.nan if e is None else float(e) for e in x], np.float64)
    na = int(np.isnan(v).sum())
    f = v[~np.isnan(v)]
    names = ["Min.", "1st Qu.", "Median", "Mean", "3rd Qu.", "Max."]
    if f.size == 0:
        vals = [None, None, None, float("nan"), None, None]
    else:
        q = np.quantile(f, [0, 0.25, 0.5, 0.75, 1.0])
        vals = [float(q[0]), float(q[1]), float(q[2]), float(f.mean()), float(q[3]), float(q[4])]
    return names, vals, na


def summary_lines(x, digits=4, width=80):
    """The lines of print(summary(x)) (print.summaryDefault, then print.table
    of a named character vector: one column width for all, right-aligned,
    each entry followed by a space, wrapped at `width`)."""
    names, vals, na = r_summary(x)
    zv = _zapsmall([v if v is not None else float("nan") for v in vals], digits + 1)
    zv = [None if vals[i] is None else zv[i] for i in range(len(vals))]  # NA stays NA, NaN (mean) NaN
    cells = r_format(zv, digits)
    if na:
        names, cells = names + ["NA's"], cells + [str(na)]
    w = max(max(len(n) for n in names), max(len(c) for c in cells))
    per = max(1, (width + 1) // (w + 1))
    lines = []
    for i in range(0, len(names), per):
        lines.append("".join(n.rjust(w) + " " for n in names[i:i + per]))
        lines.append("".join(c.rjust(w) + " " for c in cells[i:i + per]))
    return lines


class RunLog:
    """log_open / log_print / log_close of logr for NanoTel's run.log."""

    def __init__(self, save_path, t0=None, versions=""):
        self.dir = os.path.join(save_path, "log")
        os.makedirs(self.dir, exist_ok=True)
        self.path = os.path.join(self.dir, "run.log")
        self._f = open(self.path, "w")
        u = platform.uname()
        try:
            user = getpass.getuser()
        except Exception:  # noqa: BLE001
            user = str(os.getuid())
        self._f.write(RULE + "\n")
        self._f.write(f"Log Path: {os.path.abspath(self.path)} \n")
        self._f.write(f"Working Directory: {os.getcwd()} \n")
        self._f.write(f"User Name: {user} \n")
        self._f.write(f"R Version: (none: nanotel-mi355x, HIP/gfx950 hot path) \n")
        self._f.write(f"Machine: {u.node} {u.machine} \n")
        self._f.write(f"Operating System: {u.system} {u.release} {u.version} \n")
        self._f.write(f"Base Packages: {versions} \n")
        self._f.write(f"Log Start Time: {r_time(t0)} \n")
        self._f.write(RULE + "\n")
        self._f.write("\n")

    def print(self, text):
        self._f.write(f"{text} \n\n")

    def summary(self, x):
        for ln in summary_lines(x):
            self._f.write(ln + "\n")
        self._f.write("\n")

    def close(self):
        self._f.close()
