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
