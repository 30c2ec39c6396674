"""Pin the CPU oracle against the reference's own verification artefacts.

Golden data (tests/golden/, produced by make_golden.py from the reference's
Example/ directory):
  * example_summary.csv: 40 numeric cells, produced by the 2023 code version
    (no search_left/right_patterns edge extension) -> oracle legacy mode.
  * example_window_counts.json: all 1,974 window densities of P1/P2 decoded
    from the EPS plots.
  * NanoTel.R:277-302 documents a Biostrings known answer for out-of-bound
    matches (ATGG vs AATGCGCGTGGATATG, max.mismatch=1).
"""
import csv
import json
import os

import pytest

import _oracle as O

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def _example():
    names, seqs = O.read_fasta(os.path.join(GOLD, "sample.fasta"))
    rows = list(csv.DictReader(open(os.path.join(GOLD, "example_summary.csv"))))
    wins = json.load(open(os.path.join(GOLD, "example_window_counts.json")))
    return names, seqs, rows, wins


def test_biostrings_oob_known_answer():
    # NanoTel.R:277-283: views 2-5 ATGC, 8-11 GTGG, 14-17 "ATG " (out of bound)
    assert O.match_pattern("ATGG", "AATGCGCGTGGATATG", k=1) == [2, 8, 14]
    assert O.match_pattern("ATGG", "AATGCGCGTGGATATG", k=0) == []


def test_example_summary_legacy_bit_exact():
    names, seqs, rows, _ = _example()
    P = O.Patterns("TTAGGG")
    assert len(rows) == 4
    for i, (nm, s) in enumerate(zip(names, seqs)):
        r = O.analyze_read(s, P, L=100, min_density=0.6, legacy_no_ext=True)
        g = rows[i]
        assert r["telomeric"]
        assert g["sequence_ID"] == nm
        assert int(g["sequence_length"]) == len(s)
        assert (r["start"][0], r["end"][0], r["width"][0]) == (
            int(g["Telomere_start"]), int(g["Telomere_end"]), int(g["Telomere_length"]))
        assert (r["start"][1], r["end"][1], r["width"][1]) == (
            int(g["Telomere_start_mismatch"]), int(g["Telomere_end_mismatch"]),
            int(g["Telomere_length_mismatch"]))
        # fp64 densities: the golden text is the shortest round-trip repr
        assert repr(r["density"][0]) == g["telo_density"]
        assert repr(r["density"][1]) == g["telo_density_mismatch"]


def test_example_window_counts_all_1974():
    names, seqs, _, wins = _example()
    P = O.Patterns("TTAGGG")
    total = 0
    for i, s in enumerate(seqs):
        r = O.analyze_read(s, P, legacy_no_ext=True, want_windows=True)
        g = wins["reads"][i]
        assert r["n_windows"] == g["n_windows"]
        assert r["win_counts"][0] == g["p1_counts"]
        assert r["win_counts"][1] == g["p2_counts"]
        total += 2 * g["n_windows"]
    assert total == 1974


def test_example_current_code_prediction():
    """Current code (with edge extension): SURVEY.md §8(c) last row.  The start
    columns move, ends and read 1 do not.  Restatement-derived (unpinned)."""
    names, seqs, rows, _ = _example()
    P = O.Patterns("TTAGGG")
    expect = {
        1: (12070, 20405, 8336, 11251, 20405, 9155),
        2: (49241, 59426, 10186, 48956, 59426, 10471),
        3: (3805, 15877, 12073, 3805, 15877, 12073),
    }
    dens = {1: ("0.9630518234165067", "0.9743309666848716"),
            2: ("0.9837031219320637", "0.9906408174959411"),
            3: ("0.9705955437753665", "0.9874927524227616")}
    for i, s in enumerate(seqs):
        r = O.analyze_read(s, P)
        if i == 0:
            assert (r["start"], r["end"]) == ([1, 1], [2976, 2981])
            continue
        e = expect[i]
        assert (r["start"][0], r["end"][0], r["width"][0], r["start"][1], r["end"][1], r["width"][1]) == e
        assert (repr(r["density"][0]), repr(r["density"][1])) == dens[i]


def test_window_split_rules():
    # split_telo: last window absorbed when shorter than L/2; n <= L/2 -> 0 windows
    assert O.window_count(2981, 100) == 30
    assert O.window_count(20410, 100) == 204
    assert O.window_count(149, 100) == 1
    assert O.window_count(150, 100) == 1
    assert O.window_count(151, 100) == 2
    assert O.window_count(50, 100) == 0
    assert O.window_count(51, 100) == 1
    assert O.window_count(1, 1) == 0  # 1 - 1 < 0.5: the only window is dropped
    assert O.window_count(2, 1) == 1


def test_pattern_parsing_errors():
    with pytest.raises(O.OracleError) as e:
        O.Patterns(" TTAGGG")  # leading whitespace -> "" token -> empty pattern
    assert e.value.code == -1
    with pytest.raises(O.OracleError) as e:
        O.Patterns("TTAGGGX")
    assert e.value.code == -2
    with pytest.raises(O.OracleError) as e:
        O.Patterns("T" * 19)
    assert e.value.code == -3
    P = O.Patterns("TTAGGG TTAGGG")
    assert P.n_pat == 1  # unique() but still a list
