"""log/run.log (NanoTel.R:2347-2427, 2510-2516, logr 1.3.4) against the
reference's own Example_output/log/run.log (tests/golden/log/run.log): the
driver's log of the Example run, with the lines the 2023 code version did not
print yet (the version line and the arguments block, NanoTel.R:2348-2369)
taken out and the times / paths masked, equals the golden's body line for
line -- the message layout (trailing space, blank line) and R's
print(summary()) tables included.  The scan is the oracle stand-in
(test_driver.OracleNanoTel); tests/test_gpu_e2e.py runs the same on the GPU."""
import os
import re
import shutil

from nanotel_amd.runlog import RULE, summary_lines

GOLD = os.path.join(os.path.dirname(__file__), "golden")
TS = re.compile(r"\d{4}-\d\d-\d\d \d\d:\d\d:\d\d\.\d{6}")
CURRENT_ONLY = ("Telomere Analyzer  version", "############### The input argumetns",
                "The sub-sequence length  is:", "The minimal density for a telomeric subseq:",
                "##################################################################")


def _body(lines):
    """Log lines after the header block (two rules), up to a footer rule."""
    i = [k for k, x in enumerate(lines) if x == RULE][1] + 1
    out = []
    for x in lines[i:]:
        if x == RULE:
            break
        out.append(x)
    return out


def _normalise(body, inp):
    out = []
    for x in body:
        if x.startswith(CURRENT_ONLY):
            continue
        x = TS.sub("<time>", x)
        if x.strip() == inp or x.endswith("/sample.fasta "):
            x = "<input> "
        out.append(x)
    # the entries dropped above leave their blank lines behind: collapse runs
    res = []
    for x in out:
        if x == "" and res and res[-1] == "":
            continue
        res.append(x)
    return res


def run_example(tmp_path, legacy=True):
    from nanotel_amd import driver
    from test_driver import OracleNanoTel
    inp = tmp_path / "sample.fasta"
    shutil.copyfile(os.path.join(GOLD, "sample.fasta"), inp)
    out = tmp_path / "out"
    real = driver.NanoTel
    try:
        driver.NanoTel = OracleNanoTel
        driver.run(str(inp), str(out), "TTAGGG", fmt="fasta", legacy_no_ext=legacy, plot=False,
                   write_reads=False, log=lambda *a: None)
    finally:
        driver.NanoTel = real
    return str(inp), out


def test_run_log_matches_example_golden(tmp_path):
    inp, out = run_example(tmp_path)
    ours = open(out / "log" / "run.log").read().split("\n")
    gold = open(os.path.join(GOLD, "log", "run.log")).read().split("\n")
    # header: the same entries in the same order
    keys = ["Log Path:", "Working Directory:", "User Name:", "R Version:", "Machine:", "Operating System:",
            "Base Packages:", "Log Start Time:"]
    assert ours[0] == RULE and gold[0] == RULE
    for k, key in enumerate(keys):
        assert ours[1 + k].startswith(key) and gold[1 + k].startswith(key), (key, ours[1 + k])
        assert ours[1 + k].endswith(" ")
    assert ours[9] == RULE and TS.search(ours[8])
    assert ours[1].endswith(os.path.join("out", "log", "run.log") + " ")
    # body: the reference's lines, in order
    assert _normalise(_body(ours), inp) == _normalise(_body(gold), inp)
    # the current code version's extra lines (NanoTel.R:2348-2369), in logr's layout
    body = _body(ours)
    assert body[:6] == ["", "Telomere Analyzer  version v1.1.9-beta 2026-02-19 ", "", body[3], "",
                        "############### The input argumetns for this run: ################ "]
    assert "The sub-sequence length  is: 100 " in body and "The minimal density for a telomeric subseq: 0.6 " in body
    # log_close(footer = FALSE) (NanoTel.R:2514): the file ends after "Work ended at"
    assert body[-3].startswith("Work ended at: ") and body[-2:] == ["", ""]


def test_r_summary_print_layout():
    assert summary_lines([2981, 20410, 59430, 15880]) == [
        "   Min. 1st Qu.  Median    Mean 3rd Qu.    Max. ", "   2981   12655   18145   24675   30165   59430 "]
    assert summary_lines([1, 2, None]) == [
        "   Min. 1st Qu.  Median    Mean 3rd Qu.    Max.    NA's ", "   1.00    1.25    1.50    1.50    1.75    2.00       1 "]
