"""The documents cite evidence that exists: every `profiles/…`, `tools/…`, `tests/…`, `oracle/…`, `include/…` and
`fmi_amd/…` path named in DESIGN.md, INTEGRATION.md, README.md and profiles/INDEX.md must match at least one file
of the tree (a `*` in a cited name is a glob), or be a file of the reference that the text cites as such. Catches
numbers whose evidence was moved or deleted."""
import glob
import os
import re

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
DOCS = ["DESIGN.md", "INTEGRATION.md", "README.md", "profiles/INDEX.md"]
PATH = re.compile(r"(?<![\w/.])((?:profiles|tools|tests|oracle|include|fmi_amd)/[\w./*{},-]+)")
REF = "/root/reference"  # read only as a list of its files, to tell a reference citation from a missing file
REF_ONLY = ("include/comm/", "include/utils/", "include/Communicator.h", "include/fmi.h", "tests/channels.cpp",
            "tests/communicator.cpp")
# cited in the documents on purpose although not in the tree: removed tools whose history the text points to,
# and outputs of a local build (gitignored)
NOT_IN_TREE = {"tools/microbench_scan_lds.hip", "oracle/_ref/libfmi_ref.so", "fmi_amd/lib/libfmi_dev.so"}


def _expand(p):
    """`a_{x,y}.csv` -> [`a_x.csv`, `a_y.csv`]"""
    m = re.search(r"\{([^{}]*)\}", p)
    if not m:
        return [p]
    return [q for alt in m.group(1).split(",") for q in _expand(p[:m.start()] + alt + p[m.end():])]


def _cited(doc):
    text = open(os.path.join(ROOT, doc), encoding="utf-8").read()
    for raw in PATH.findall(text):
        p = raw.rstrip(".,:;)`")
        if p.endswith("/"):
            continue
        yield p


@pytest.mark.parametrize("doc", DOCS)
def test_cited_paths_exist(doc):
    base = os.path.dirname(os.path.join(ROOT, doc)) if doc.startswith("profiles/") else ROOT
    missing = []
    for p in _cited(doc):
        if p in NOT_IN_TREE or p.split(":")[0] in NOT_IN_TREE:
            continue
        p = p.split(":")[0]  # file:line citations
        if any(glob.glob(os.path.join(ROOT, q)) or glob.glob(os.path.join(base, q)) for q in _expand(p)):
            continue
        if os.path.isdir(REF) and any(glob.glob(os.path.join(REF, q)) for q in _expand(p)):
            continue  # a file of the reference (include/Communicator.h, tests/channels.cpp, ...), cited as such
        if not os.path.isdir(REF) and p.startswith(REF_ONLY):
            continue  # no reference checkout here to look in
        if doc.startswith("profiles/") and glob.glob(os.path.join(ROOT, "profiles", "archive", os.path.basename(p))):
            continue
        missing.append(p)
    assert not missing, f"{doc} cites paths that do not exist: {sorted(set(missing))}"


DRIVER = re.compile(r"(?<![\w/.])((?:BENCH|GPUTEST|SCALE|MULTICHIP)_r\d\d\.json)")


@pytest.mark.parametrize("doc", DOCS)
def test_cited_driver_records_exist(doc):
    """every driver record a document cites (BENCH_r0N.json, GPUTEST_r0N.json, SCALE_…,
    MULTICHIP_…) is in the tree; a result quoted from a record that is not there cannot be checked."""
    text = open(os.path.join(ROOT, doc), encoding="utf-8").read()
    missing = sorted({r for r in DRIVER.findall(text) if not os.path.exists(os.path.join(ROOT, r))})
    assert not missing, f"{doc} cites driver records that do not exist: {missing}"


# ---- figures quoted from the line's cpu_baseline and c5 blocks -----------------------------
NUM = re.compile(r"(?<![\w.])(\d{1,3}(?:,\d{3})+(?:\.\d+)?|\d+\.\d+)(?![\w.]*\d)")
QUOTES = re.compile(r"cpu_baseline|(?<![\w/-])c5(?:[._]|\b)")
RECORD_GLOBS = ["BENCH_r0*.json", "profiles/*.json", "profiles/*.jsonl", "profiles/*.log", "profiles/*.txt",
                "profiles/*.csv", "profiles/archive/*"]


def _record_figures():
    """Every decimal figure in a committed record, at every rounding from its own precision down to 0 places."""
    out = set()
    for g in RECORD_GLOBS:
        for path in glob.glob(os.path.join(ROOT, g)):
            if not os.path.isfile(path):
                continue
            text = open(path, encoding="utf-8", errors="replace").read()
            for m in re.finditer(r"-?\d+(?:\.\d+)?(?:[eE][-+]?\d+)?", text):
                v = float(m.group(0))
                mant = m.group(0).split("e")[0].split("E")[0]
                digits = len(mant.split(".")[1]) if "." in mant else 0
                for d in range(0, digits + 1):
                    out.add(f"{abs(v):.{d}f}")
                for d in range(0, 3):  # kernel traces hold ns: the same figure in µs or ms
                    out.add(f"{abs(v) / 1e3:.{d}f}")
                    out.add(f"{abs(v) / 1e6:.{d}f}")
    return out


def _segments(text):
    """Table rows one by one, other text by paragraph."""
    for block in re.split(r"\n\s*\n", text):
        lines = block.splitlines()
        if lines and all(x.lstrip().startswith("|") for x in lines):
            yield from lines
        else:
            yield " ".join(lines)


@pytest.mark.parametrize("doc", ["DESIGN.md", "INTEGRATION.md"])
def test_quoted_cpu_baseline_and_c5_figures_match_a_record(doc):
    """A sentence (paragraph or table row) that names the line's `cpu_baseline` or `c5` blocks may quote only decimal
    figures found in a committed record (BENCH_r0N.json, profiles/…), at the precision quoted: a number that no
    record holds is a transcription error or a figure whose evidence is gone."""
    figures = _record_figures()
    bad = []
    for seg in _segments(open(os.path.join(ROOT, doc), encoding="utf-8").read()):
        if not QUOTES.search(seg):
            continue
        for raw in NUM.findall(seg):
            f = raw.replace(",", "")
            if "." not in f:
                continue
            if f not in figures:
                bad.append((f, seg[:120]))
    assert not bad, f"{doc} quotes figures no committed record holds: {bad}"
