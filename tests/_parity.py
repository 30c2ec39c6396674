"""Shared helpers: compare the HIP path (nanotel_amd) with the CPU oracle."""
import math

import _oracle as O


def oracle_rows(seqs, patterns, tvr=None, L=100, min_density=0.6, right_edge=False, rc=False,
                legacy=False, want_windows=True, want_hits=True):
    P = O.Patterns(patterns, tvr)
    rows = []
    for s in seqs:
        if rc:
            s = O.reverse_complement(s)
        rows.append(O.analyze_read(s, P, L=L, min_density=min_density, right_edge=right_edge,
                                   legacy_no_ext=legacy, want_windows=want_windows, want_hits=want_hits))
    return rows


def compare(nt, res, orows, check_windows=True, check_hits=True):
    """Assert bit-exact agreement; returns the number of reads compared."""
    bad = []
    for i, o in enumerate(orows):
        npass = o["n_pass"]
        g_start = [int(x) for x in res["start"][i][:npass]]
        g_end = [int(x) for x in res["end"][i][:npass]]
        g_den = [float(x) for x in res["density"][i][:npass]]
        if g_start != o["start"] or g_end != o["end"]:
            bad.append((i, "range", g_start, g_end, o["start"], o["end"]))
            continue
        for p in range(npass):
            od, gd = o["density"][p], g_den[p]
            if not (od == gd or (math.isnan(od) and math.isnan(gd))):
                bad.append((i, "density", p, repr(gd), repr(od)))
        if bool(res["telomeric"][i]) != o["telomeric"]:
            bad.append((i, "telomeric", bool(res["telomeric"][i]), o["telomeric"]))
        if check_windows:
            for p in range(npass):
                g = [int(x) for x in nt.window_counts(res, i, p)]
                if g != o["win_counts"][p]:
                    diff = [j for j in range(len(g)) if g[j] != o["win_counts"][p][j]][:5]
                    bad.append((i, "windows", p, diff))
        if check_hits and "hits" in o:
            g = [int(x) for x in res["hits"][i]]
            if g != o["hits"]:
                bad.append((i, "hits", g, o["hits"]))
    assert not bad, f"{len(bad)} mismatches, first: {bad[:5]}"
    return len(orows)
