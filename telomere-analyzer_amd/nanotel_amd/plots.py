"""Single-read density plots: plot_single_telo_with_gray_area
and plot_single_telo_with_tvr of NanoTel.R:1271-1624, called per telomeric read
(NanoTel.R:1876-1912):

    single_read_plots/read<serial>.jpeg      x axis up to max_length (1e5)
    single_read_plots_adj/read<serial>.jpeg  x axis up to the read length
    single_read_plots_adj/read<serial>.eps   the same, setEPS(); postscript()

The figure is R base graphics: plot(type = "n") with xlim c(1, x_length +
round(x_length / 4.15)), ylim c(0, 1); axis(1) every 1 kb ("%.1fkb"),
title(xlab = "Position", adj = 0), axis(2, las = 2); one density polygon per
pass (TVR pass orange3, mismatch pass orange, exact pass salmon) through
(1, 0), (window start, density)..., (n, last density), (n, 0); red / blue /
yellow(3) rectangles under the axis for the called telomere, sub-telomere and
the mismatch (TVR) extensions; dashed lines at 0 and 1; legend(x_length, 1);
title(main, sub, ylab = "Density").

The EPS writer restates what R's postscript() device emits for that figure:
the layout arithmetic of the graphics engine (default par: 7 in square
device, mar c(5.1, 4.1, 4.1, 2.1), mgp c(3, 1, 0), tcl -0.5, 4 % axis
extension, yLineBias 0.2, text centred on half the ascent of "M"), axis
label thinning (a label is drawn when it starts at least one "m" width after
the previous drawn one), legend() geometry, and the device's output (graphics
state emitted on change and after every clip, 2-decimal coordinates, relative
"dx dy l" moves with an absolute lineto every 100th polygon point, Helvetica
widths with kerning, kerned strings split into "ta"/"tb" pieces).  The
Example plots of the reference are reproduced byte for byte
(tests/test_plots.py).  The JPEGs draw the same layout on a 750 x 300 pixel
canvas (jpeg(width = 750, height = 300), pointsize 12 at 72 dpi) with PIL;
they are not pixel-identical to R's rasteriser.
"""
import math
import os

import numpy as np

from . import _psdata as F

# colours (R's colour table, 0-255)
RED, BLUE, YELLOW, YELLOW3 = (255, 0, 0), (0, 0, 255), (255, 255, 0), (205, 205, 0)
SALMON, ORANGE, ORANGE3, BLACK = (250, 128, 114), (255, 165, 0), (205, 133, 0), (0, 0, 0)

MAX_LENGTH = 1e5                 # search_patterns(max_length = 1e5), NanoTel.R:2001
TITLE = "Telomeric repeat density"  # analyze_read's title (NanoTel.R:2059)
_LH = 14.4                       # one margin line (cex 1, ps 12, mex 1): 0.2 in
_MAR = (5.1, 4.1, 4.1, 2.1)      # bottom, left, top, right
_BIAS = 0.2                      # yLineBias of the device


def _font(face):
    return (F.PLAIN_WIDTHS, F.PLAIN_KERN, F.PLAIN_ASCENT_M) if face == 1 else \
        (F.BOLD_WIDTHS, F.BOLD_KERN, F.BOLD_ASCENT_M)


def _w(c, widths):
    o = ord(c)
    return widths[o - 32] if 32 <= o <= 126 else widths[0]


def str_width(s, face, size, kern=True):
    """Width in points of s at an integer font size (PostScriptStringWidth)."""
    widths, pairs, _ = _font(face)
    tot = sum(_w(c, widths) for c in s)
    if kern:
        tot += sum(pairs.get((ord(a), ord(b)), 0.0) for a, b in zip(s, s[1:]))
    return 0.001 * size * tot


def _fsize(cex):
    return int(math.floor(cex * 12 + 0.5))


# ---------------------------------------------------------------- the figure


class _Figure:
    """Device geometry of one plot: W x H points, user x range from x_length."""

    def __init__(self, W, H, x_length):
        self.W, self.H = float(W), float(H)
        # plt (NFC) from the margins in inches over the 7 in (or W/72 in) figure
        self.plt = (_MAR[1] * 0.2 * 72 / self.W, 1 - _MAR[3] * 0.2 * 72 / self.W,
                    _MAR[0] * 0.2 * 72 / self.H, 1 - _MAR[2] * 0.2 * 72 / self.H)
        xmax = x_length + round(x_length / 4.15)  # R's round(): half to even, like Python's
        d = (xmax - 1) * 0.04
        self.usr = (1 - d, xmax + d, 0 - 0.04, 1 + 0.04)
        self.bx = (self.plt[1] - self.plt[0]) / (self.usr[1] - self.usr[0])
        self.ax = self.plt[0] - self.usr[0] * self.bx
        self.by = (self.plt[3] - self.plt[2]) / (self.usr[3] - self.usr[2])
        self.ay = self.plt[2] - self.usr[2] * self.by

    def nfc_x(self, x):
        return self.ax + x * self.bx

    def X(self, x):
        return self.nfc_x(x) * self.W

    def Y(self, y):
        return (self.ay + y * self.by) * self.H

    @property
    def left(self):
        return self.plt[0] * self.W

    @property
    def right(self):
        return self.plt[1] * self.W

    @property
    def bottom(self):
        return self.plt[2] * self.H

    @property
    def top(self):
        return self.plt[3] * self.H

    def xinch(self):  # user x units per inch
        return (self.usr[1] - self.usr[0]) / ((self.right - self.left) / 72.0)

    def yinch(self):
        return (self.usr[3] - self.usr[2]) / ((self.top - self.bottom) / 72.0)


def _ops(fig, x_length, seq_length, passes, rects, legend, sub_title):
    """The drawing as device operations (what the graphics engine hands the
    device), in R's call order.  passes: [(fill colour, xs, ys)] drawn in
    order; rects: [(x0, x1, colour)] (user x, y from -0.1 to 0)."""
    ops = []
    add = ops.append
    dev_clip = (0.0, 0.0, fig.W, fig.H)
    plot_clip = (fig.left, fig.bottom, fig.right, fig.top)
    lwd1 = dict(lwd=1.0, lty=0)
    # plot(type = "n"): the box
    add(("clip", dev_clip))
    add(("polygon", [fig.left, fig.right, fig.right, fig.left], [fig.bottom, fig.bottom, fig.top, fig.top],
         None, BLACK, lwd1))
    # axis(1, at = seq(1, x_length, by = 1000), labels = sprintf("%.1fkb", at / 1000))
    add(("clip", dev_clip))
    add(("clip", dev_clip))
    at = list(range(1, int(x_length) + 1, 1000))
    lo, hi = fig.usr[0], fig.usr[1]
    at = [a for a in at if lo <= a <= hi]
    if at:
        add(("line", fig.X(at[0]), fig.bottom, fig.X(at[-1]), fig.bottom, BLACK, lwd1))
        for a in at:
            add(("line", fig.X(a), fig.bottom, fig.X(a), fig.bottom - 0.5 * _LH, BLACK, lwd1))
        gap = str_width("m", 1, 12) / fig.W
        tlast = -1.0
        ybase = fig.bottom - (1 + 1 - _BIAS) * _LH
        for a in at:
            lab = "%.1fkb" % (a / 1000.0)
            temp = fig.nfc_x(a)
            labw = str_width(lab, 1, 12) / fig.W
            if temp - 0.5 * labw - tlast >= gap:
                add(("text", fig.X(a), ybase, lab, 0.5, 0, 1, 1.0, BLACK))
                tlast = temp + 0.5 * labw
    # title(xlab = "Position", adj = 0)
    add(("clip", dev_clip))
    add(("text", fig.left, fig.bottom - (3 + 1 - _BIAS) * _LH, "Position", 0.0, 0, 1, 1.0, BLACK))
    # axis(2, at = seq(-0.1, 1, by = 0.1), las = 2)
    add(("clip", dev_clip))
    yat = [-0.1 + k * 0.1 for k in range(12)]
    inside = [(k, v) for k, v in enumerate(yat) if fig.usr[2] <= v <= fig.usr[3]]
    add(("line", fig.left, fig.Y(max(yat[0], fig.usr[2])), fig.left, fig.Y(min(yat[-1], fig.usr[3])), BLACK, lwd1))
    for _, v in inside:
        add(("line", fig.left, fig.Y(v), fig.left - 0.5 * _LH, fig.Y(v), BLACK, lwd1))
    asc = 0.001 * F.PLAIN_ASCENT_M * 12
    for k, v in inside:
        add(("text", fig.left - 1 * _LH, fig.Y(v) - 0.5 * asc, "%.1f" % ((k - 1) / 10.0), 1.0, 0, 1,
             1.0, BLACK))
    # the density polygons, rectangles, ablines and legend (clipped to the plot)
    add(("clip", plot_clip))
    for col, xs, ys in passes:
        px = [fig.X(1)] + [fig.X(x) for x in xs] + [fig.X(seq_length), fig.X(seq_length)]
        py = [fig.Y(0)] + [fig.Y(y) for y in ys] + [fig.Y(ys[-1] if ys else float("nan")), fig.Y(0)]
        add(("polygon", px, py, col, BLACK, dict(lwd=0.5, lty=0)))
    for x0, x1, col in rects:
        add(("rect", fig.X(x0), fig.Y(-0.1), fig.X(x1), fig.Y(0), col, BLACK, lwd1))
    dashed = dict(lwd=1.0, lty=0x44)
    add(("line", fig.left, fig.Y(1), fig.right, fig.Y(1), BLACK, dashed))
    add(("line", fig.left, fig.Y(0), fig.right, fig.Y(0), BLACK, dashed))
    _legend(fig, x_length, legend, add)
    # title(main = title, sub = sub_title, ylab = "Density")
    add(("clip", dev_clip))
    cx = 0.5 * (fig.left + fig.right)
    asc_main = 0.001 * F.BOLD_ASCENT_M * _fsize(1.2)
    add(("text", cx, fig.top + 0.5 * _MAR[2] * _LH - 0.5 * asc_main, TITLE, 0.5, 0, 2, 1.2, BLACK))
    add(("text", cx, fig.bottom - (3 + 1 + 1 - _BIAS) * _LH, sub_title, 0.5, 0, 1, 1.0, BLACK))
    add(("text", fig.left - (3 + _BIAS) * _LH, 0.5 * (fig.bottom + fig.top), "Density", 0.5, 90, 1, 1.0, BLACK))
    return ops


def _legend(fig, x, entries, add):
    """legend(x, y = 1, legend, col, lty = 1, lwd = 2, cex = 1.2) geometry
    (graphics::legend, xjust 0, yjust 1, seg.len 2, x.intersp 1)."""
    cex = 1.2
    size = _fsize(cex)
    xc = cex * 0.15 * fig.xinch()   # Cex * xinch(cin[1])
    yc = cex * 0.2 * fig.yinch()    # Cex * yinch(cin[2])
    upt_x = fig.xinch() / 72.0
    text_width = max(str_width(s, 1, size) for s, _ in entries) * upt_x
    asc = 0.001 * F.PLAIN_ASCENT_M * size * fig.yinch() / 72.0
    ymax = yc * max(1.0, asc / yc)
    ychar = ymax
    w0 = text_width + 2 * xc + 2 * xc
    w = w0 + 0.5 * xc
    h = len(entries) * ychar + yc
    left, top = float(x), 1.0
    add(("rect", fig.X(left), fig.Y(top), fig.X(left + w), fig.Y(top - h), None, BLACK, dict(lwd=1.0, lty=0)))
    xt = left + xc
    for i, (s, col) in enumerate(entries):
        yt = top - ymax - i * ychar
        add(("line", fig.X(xt), fig.Y(yt), fig.X(xt + 2 * xc), fig.Y(yt), col, dict(lwd=2.0, lty=0)))
    asc_dev = 0.001 * F.PLAIN_ASCENT_M * size
    for i, (s, _) in enumerate(entries):
        yt = top - ymax - i * ychar
        add(("text", fig.X(xt + 3 * xc), fig.Y(yt) - 0.5 * asc_dev, s, 0.0, 0, 1, cex, BLACK))


# ---------------------------------------------------------------- EPS output


def _col(c):
    def one(v):
        v = v / 255.0
        return "0" if v == 0 else ("1" if v == 1 else "%.4f" % v)
    return " ".join(one(v) for v in c) + " srgb"


def _ps_string(s):
    out = []
    for ch in s:
        o = ord(ch)
        if ch in "()\\":
            out.append("\\" + ch)
        elif 32 <= o <= 126:
            out.append(ch)
        else:
            out.append("\\%03o" % (o & 0xFF))
    return "(" + "".join(out) + ")"


def _rline(x0, y0, x1, y1):
    x = round(x1, 2) - round(x0, 2)
    y = round(y1, 2) - round(y0, 2)
    xs = "0" if abs(x) < 0.005 else "%.2f" % x
    ys = " 0" if abs(y) < 0.005 else " %.2f" % y
    return xs + ys + " l\n"


class _PS:
    """R's postscript() device state machine: colour, fill, line style and
    font are written when they change, and all of them again after a clip
    (which is a grestore/gsave)."""

    def __init__(self):
        self.o = []
        self.invalidate()

    def invalidate(self):
        self.col = self.fill = self.font = None
        self.lwd = self.lty = None
        self.style = False

    def clip(self, r):
        self.o.append("%.2f %.2f %.2f %.2f cl\n" % r)
        self.invalidate()

    def set_col(self, c):
        if c != self.col:
            self.col = c
            self.o.append(_col(c) + "\n")

    def set_fill(self, c):
        if c != self.fill:
            self.fill = c
            self.o.append("/bg { " + _col(c) + " } def\n")

    def set_line(self, st):
        lwd, lty = st["lwd"], st["lty"]
        if lwd != self.lwd or lty != self.lty:
            self.lwd, self.lty = lwd, lty
            self.o.append("%.2f setlinewidth\n" % (lwd * 0.75))
            dash = []
            t = lty
            while t & 15 and len(dash) < 8:
                dash.append(t & 15)
                t >>= 4
            lw = lwd * 0.75
            a = 1.0  # round line ends (lend = 0 -> setlinecap 1)
            parts = ["%.2f" % (lw * (d + a if i % 2 else d - a)) for i, d in enumerate(dash)]
            self.o.append("[" + "".join(" " + p for p in parts) + "] 0 setdash\n")
        if not self.style:
            self.style = True
            self.o.append("1 setlinecap\n1 setlinejoin\n10.00 setmiterlimit\n")

    def set_font(self, face, size):
        if (face, size) != self.font:
            self.font = (face, size)
            self.o.append("/Font%d findfont %d s\n" % (face, size))

    def polygon(self, xs, ys, fill, col, st):
        code = (2 if fill is not None else 0) + (1 if col is not None else 0)
        if fill is not None:
            self.set_fill(fill)
        if col is not None:
            self.set_col(col)
            self.set_line(st)
        o = self.o
        o.append("np\n")
        o.append(" %.2f %.2f m\n" % (xs[0], ys[0]))
        for i in range(1, len(xs)):
            if i % 100 == 0:
                o.append("%.2f %.2f lineto\n" % (xs[i], ys[i]))
            else:
                o.append(_rline(xs[i - 1], ys[i - 1], xs[i], ys[i]))
        o.append("cp p%d\n" % code)

    def line(self, x0, y0, x1, y1, col, st):
        self.set_col(col)
        self.set_line(st)
        self.o.append("np\n%.2f %.2f m\n" % (x0, y0) + _rline(x0, y0, x1, y1) + "o\n")

    def rect(self, x0, y0, x1, y1, fill, col, st):
        code = (2 if fill is not None else 0) + (1 if col is not None else 0)
        if fill is not None:
            self.set_fill(fill)
        if col is not None:
            self.set_col(col)
            self.set_line(st)
        self.o.append("%.2f %.2f %.2f %.2f r p%d\n" % (x0, y0, x1 - x0, y1 - y0, code))

    def text(self, x, y, s, hadj, rot, face, cex, col):
        size = _fsize(cex)
        self.set_font(face, size)
        self.set_col(col)
        _, pairs, _ = _font(face)
        cuts = [i for i in range(len(s) - 1) if (ord(s[i]), ord(s[i + 1])) in pairs]
        if not cuts:
            ha = {0.0: "0", 0.5: ".5", 1.0: "1"}.get(hadj, "%.2f" % hadj)
            ro = {0: "0", 90: "90"}.get(rot, "%.2f" % rot)
            self.o.append("%.2f %.2f %s %s %s t\n" % (x, y, _ps_string(s), ha, ro))
            return
        if hadj != 0:
            w = str_width(s, face, size, kern=False)
            r = rot * math.pi / 180.0
            x -= hadj * w * math.cos(r)
            y -= hadj * w * math.sin(r)
        nout = 0
        first = True
        for i in cuts:
            piece = s[nout:i + 1]
            if first:
                self.o.append("%.2f %.2f %s %d ta" % (x, y, _ps_string(piece), int(rot)))
                first = False
            else:
                self.o.append("\n%.3f %s tb" % (kx, _ps_string(piece)))
            kx = 0.001 * size * pairs[(ord(s[i]), ord(s[i + 1]))]
            nout = i + 1
        self.o.append("\n%.3f %s tb" % (kx, _ps_string(s[nout:])))
        self.o.append(" gr\n")


def render_eps(ops):
    ps = _PS()
    ps.o.append(F.PROLOG)
    ps.o.append("%%Page: 1 1\nbp\n")
    for op in ops:
        kind = op[0]
        if kind == "clip":
            ps.clip(op[1])
        elif kind == "polygon":
            ps.polygon(*op[1:])
        elif kind == "line":
            ps.line(*op[1:])
        elif kind == "rect":
            ps.rect(*op[1:])
        elif kind == "text":
            ps.text(*op[1:])
    ps.o.append("ep\n%%Trailer\n%%Pages: 1\n%%EOF\n")
    return "".join(ps.o)


# ---------------------------------------------------------------- JPEG output


_JPEG_FONTS = {}  # (face, size) -> PIL font, loaded once per process
_TEXT_SPRITES = {}  # (text, face, cex, colour, rotation, scale) -> (RGBA sprite, ascent, width), per process


def render_jpeg(ops, W, H, path, S=3):
    """Rasterise the same device operations with PIL (y flipped, 1 pt = 1 px at
    R's 72 dpi), as R's cairo jpeg() device does: anti-aliased -- drawn at S
    times the size and box-filtered down --, lines of lwd 1 = 1/96 in = 0.75 px,
    and text set to the Helvetica widths the layout was computed with (the
    DejaVu glyphs, the only TrueType face here, scaled horizontally to them;
    R's device substitutes a Helvetica-metric face)."""
    from PIL import Image, ImageDraw, ImageFont
    img = Image.new("RGB", (int(W) * S, int(H) * S), (255, 255, 255))
    dr = ImageDraw.Draw(img)
    fonts = _JPEG_FONTS

    def font(face, size):
        key = (face, size)
        if key not in fonts:
            try:
                import matplotlib
                d = os.path.join(os.path.dirname(matplotlib.__file__), "mpl-data", "fonts", "ttf")
                fonts[key] = ImageFont.truetype(os.path.join(d, "DejaVuSans-Bold.ttf" if face == 2
                                                             else "DejaVuSans.ttf"), size)
            except Exception:  # noqa: BLE001 -- any TrueType failure: PIL's bitmap font
                fonts[key] = ImageFont.load_default()
        return fonts[key]

    clip = (0.0, 0.0, W, H)

    def P(x, y):
        return (x * S, (H - y) * S)

    def width(st):
        return max(1, int(round(0.75 * S * st.get("lwd", 1.0))))

    def inside(x0, y0, x1, y1):
        return not (max(x0, x1) < clip[0] or min(x0, x1) > clip[2] or max(y0, y1) < clip[1]
                    or min(y0, y1) > clip[3])

    def cl(x, y):
        return min(max(x, clip[0]), clip[2]), min(max(y, clip[1]), clip[3])

    for op in ops:
        kind = op[0]
        if kind == "clip":
            clip = op[1]
        elif kind == "polygon":
            xs, ys, fill, col, st = op[1:]
            # (the points clipped and scaled as arrays: the same float64
            # arithmetic as P(*cl(x, y)) point by point, a fifth of the time)
            xa, ya = np.asarray(xs, np.float64), np.asarray(ys, np.float64)
            ok = ~(np.isnan(xa) | np.isnan(ya))
            xa = np.minimum(np.maximum(xa[ok], clip[0]), clip[2]) * S
            ya = (H - np.minimum(np.maximum(ya[ok], clip[1]), clip[3])) * S
            if xa.size >= 3:
                pts = np.stack((xa, ya), axis=1).ravel().tolist()
                if fill is not None:
                    dr.polygon(pts, fill=fill)
                if col is not None:
                    dr.line(pts + pts[:2], fill=col, width=width(st), joint="curve")
        elif kind == "line":
            x0, y0, x1, y1, col, st = op[1:]
            if inside(x0, y0, x1, y1):
                wd = width(st)
                if st["lty"]:  # lty 2: 4 on, 4 off (in units of the line width * 0.75 pt)
                    ln = math.hypot(x1 - x0, y1 - y0)
                    step = 4 * 0.75 * st["lwd"]
                    t = 0.0
                    while t < ln:
                        u = min(ln, t + step)
                        dr.line([P(x0 + (x1 - x0) * t / ln, y0 + (y1 - y0) * t / ln),
                                 P(x0 + (x1 - x0) * u / ln, y0 + (y1 - y0) * u / ln)], fill=col, width=wd)
                        t += 2 * step
                else:
                    dr.line([P(x0, y0), P(x1, y1)], fill=col, width=wd)
        elif kind == "rect":
            x0, y0, x1, y1, fill, col, st = op[1:]
            (xa, ya), (xb, yb) = P(*cl(x0, y0)), P(*cl(x1, y1))
            xa, xb = sorted((xa, xb))
            ya, yb = sorted((ya, yb))
            if xb > xa or fill is not None:
                if fill is not None:
                    dr.rectangle([xa, ya, xb, yb], fill=fill)
                if col is not None:
                    dr.line([(xa, ya), (xb, ya), (xb, yb), (xa, yb), (xa, ya)], fill=col, width=width(st))
        elif kind == "text":
            x, y, s, hadj, rot, face, cex, col = op[1:]
            key = (s, face, cex, col, rot, S)
            hit = _TEXT_SPRITES.get(key)
            if hit is None:  # the string set at the Helvetica width once a process (tick labels, titles, legend)
                size = _fsize(cex)
                f = font(face, size * S)
                target = max(1, int(round(str_width(s, face, size) * S)))  # Helvetica width, px
                asc, desc = f.getmetrics()
                tmp = Image.new("RGBA", (int(dr.textlength(s, font=f)) + 2, asc + desc), (255, 255, 255, 0))
                ImageDraw.Draw(tmp).text((0, asc), s, font=f, fill=col, anchor="ls")
                tmp = tmp.resize((target, tmp.height), Image.BILINEAR)
                if rot == 90:
                    tmp = tmp.rotate(90, expand=True)
                if len(_TEXT_SPRITES) >= 8192:
                    _TEXT_SPRITES.clear()
                hit = _TEXT_SPRITES[key] = (tmp, asc, target)
            tmp, asc, target = hit
            bx, by = P(x, y)
            if rot == 90:
                img.paste(tmp, (int(round(bx - asc)), int(round(by - (1.0 - hadj) * target))), tmp)
            else:
                img.paste(tmp, (int(round(bx - hadj * target)), int(round(by - asc))), tmp)
    # box filter down to the device size (reduce: the same S x S averages as
    # resize(BOX), rounded within 1 of it, 4x faster)
    img = img.reduce(S) if img.size == (int(W) * S, int(H) * S) else img.resize((int(W), int(H)), Image.BOX)
    img.save(path, "JPEG", quality=75)


# ---------------------------------------------------------------- the plots


def figure_spec(seq_length, subs, subs_mm, seq_start, seq_end, gray_start, gray_end, subs_tvr=None,
                tvr_start=-1, tvr_end=-1):
    """Rectangles, legend entries and sub-title of plot_single_telo_with_gray_area
    (NanoTel.R:1339-1408) or, with subs_tvr, plot_single_telo_with_tvr
    (NanoTel.R:1473-1622).  subs* = (window starts, densities)."""
    n = seq_length
    tvr = subs_tvr is not None
    rects = []
    if tvr:
        legend = [("telomere", RED), ("gray area", YELLOW), ("tvr", YELLOW3), ("sub-telomere", BLUE),
                  ("Density", SALMON), ("Density MM", ORANGE), ("DensMM+TVRs", ORANGE3)]
    else:
        legend = [("telomere", RED), ("gray area", YELLOW), ("sub-telomere", BLUE), ("Density", SALMON),
                  ("Density MM", ORANGE)]
    tl = lambda a, b: abs(a - b) + 1  # noqa: E731
    if seq_start > -1:
        rects.append((seq_start, seq_end, RED))
        rects.append((seq_end + 1, n, BLUE))
        if seq_start > 1:
            rects.append((1, seq_start, BLUE))
        if gray_start == -1:
            if not tvr:
                sub = (f"Read length: {n} , Telomere length: {tl(seq_start, seq_end)} , "
                       "Faild to calculate Telomere length with mismatches")
                return rects, legend, sub
            if tvr_start == -1:
                sub = (f"Read length: {n} , Telomere length: {tl(seq_start, seq_end)} , "
                       "Faild to calculate Telomere length with mismatches/tvr")
                return rects, legend, sub
            if tvr_start < seq_start:
                rects.append((tvr_start, seq_start, YELLOW3))
            if tvr_end > seq_end:
                rects.append((seq_end, tvr_end, YELLOW3))
            sub = (f"Read length: {n} , Telomere length: {tl(seq_start, seq_end)} , "
                   f"Faild to calculate Telomere length with mismatches Telomere length with tvr: "
                   f"{tl(tvr_start, tvr_end)}")
            return rects, legend, sub
        if gray_start < seq_start:
            rects.append((gray_start, seq_start, YELLOW))
        if gray_end > seq_end:
            rects.append((seq_end, gray_end, YELLOW))
        if tvr and tvr_start != -1:
            if gray_start > tvr_start:
                rects.append((tvr_start, gray_start, YELLOW3))
            if gray_end < tvr_end:
                rects.append((gray_end, tvr_end, YELLOW3))
    else:
        rects.append((gray_start, gray_end, YELLOW))
        rects.append((gray_end + 1, n, BLUE))
        if gray_start > 1:
            rects.append((1, gray_start, BLUE))
        if tvr and tvr_start != -1:
            if gray_start > tvr_start:
                rects.append((tvr_start, gray_start, YELLOW3))
            if gray_end < tvr_end:
                rects.append((gray_end, tvr_end, YELLOW3))
    telo = ", No telomere length" if seq_start == -1 else f", Telomere length: {tl(seq_start, seq_end)}"
    sub = f"Read length: {n} {telo} , Telomere length with mismatches: {tl(gray_start, gray_end)}"
    if tvr:
        if tvr_start != -1:
            sub += f" , with mismatch+tvr: {tl(tvr_start, tvr_end)}"
        else:
            sub += " , failed to calculate Telomere length with mismatch+tvr"
    return rects, legend, sub


def plot_ops(x_length, seq_length, subs, subs_mm, seq_start, seq_end, gray_start, gray_end, W=504, H=504,
             subs_tvr=None, tvr_start=-1, tvr_end=-1):
    fig = _Figure(W, H, x_length)
    rects, legend, sub = figure_spec(seq_length, subs, subs_mm, seq_start, seq_end, gray_start, gray_end,
                                     subs_tvr, tvr_start, tvr_end)
    passes = []
    if subs_tvr is not None:
        passes.append((ORANGE3, subs_tvr[0], subs_tvr[1]))
    passes += [(ORANGE, subs_mm[0], subs_mm[1]), (SALMON, subs[0], subs[1])]
    return _ops(fig, x_length, seq_length, passes, rects, legend, sub)


def window_table(n, L, counts):
    """(start_index, density) of analyze_subtelos' windows (split_telo,
    NanoTel.R:199-227; density = count / width in fp64, get_sub_density)."""
    nw = len(counts)
    starts = [1 + k * L for k in range(nw)]
    dens = [int(counts[k]) / (L if k < nw - 1 else n - starts[k] + 1) for k in range(nw)]
    return starts, dens


def write_read_plots(save_path, serial_text, seq_length, subs, subs_mm, seq_start, seq_end, gray_start, gray_end,
                     subs_tvr=None, tvr_start=-1, tvr_end=-1, jpeg=True):
    """The three files analyze_read writes per telomeric read (NanoTel.R:1876-1912)."""
    args = (seq_length, subs, subs_mm, seq_start, seq_end, gray_start, gray_end)
    kw = dict(subs_tvr=subs_tvr, tvr_start=tvr_start, tvr_end=tvr_end)
    adj = os.path.join(save_path, "single_read_plots_adj")
    full = os.path.join(save_path, "single_read_plots")
    if jpeg:
        render_jpeg(plot_ops(MAX_LENGTH, *args, W=750, H=300, **kw), 750, 300,
                    os.path.join(full, f"read{serial_text}.jpeg"))
        render_jpeg(plot_ops(seq_length, *args, W=750, H=300, **kw), 750, 300,
                    os.path.join(adj, f"read{serial_text}.jpeg"))
    with open(os.path.join(adj, f"read{serial_text}.eps"), "w") as f:
        f.write(render_eps(plot_ops(seq_length, *args, **kw)))
