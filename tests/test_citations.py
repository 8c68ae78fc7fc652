"""Every `Networks.py:N` / `Blocks.py:N` / `main.py:N` citation in the product, the oracle and the
docs points at a line that exists, and the key ones point at the symbol they name.

Reads /root/reference as text (study only); skipped where the reference is absent (the GPU box)."""
from __future__ import annotations

import re
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parents[1]
REF = Path("/root/reference/src")
pytestmark = pytest.mark.skipif(not REF.exists(), reason="reference sources not present")

CITING = [
    *ROOT.glob("spwgnn_amd/*.py"), *ROOT.glob("spwgnn_amd/csrc/*"), *ROOT.glob("oracle/*.py"),
    *ROOT.glob("include/*.h"), ROOT / "DESIGN.md", ROOT / "INTEGRATION.md", ROOT / "README.md", *ROOT.glob("tools/*.py"),
    ROOT / "bench.py", *ROOT.glob("tests/*.py"),
]
FILES = ("Networks", "Blocks", "main", "JengaBuilder", "TowerCreator", "DataGenerator")
ANCHOR = re.compile(r"\b(" + "|".join(FILES) + r")\.py:")
# the numbers right after the anchor, with ", N", "/N", ", :N", " / :N" continuations
LEAD = re.compile(r"(\d+)(?:-\d+)?(?:\s*[,/]\s*:?\d+(?:-\d+)?)*")
# a bare ":N" later on the same line, before the next file anchor, cites the same file
BARE = re.compile(r"(?<![\w.:/]):(\d+)(?:-(\d+))?")


def _lines(name):
    return (REF / f"{name}.py").read_text().splitlines()


def cited_lines(line: str):
    """(file, [line numbers]) for every reference citation on one line of text, following the
    continuations after the `File.py:` anchor (`Networks.py:35-37, 58-71`, `:29 / :80`, and a later
    bare `:88` on the same line)."""
    out = []
    anchors = list(ANCHOR.finditer(line))
    for i, m in enumerate(anchors):
        seg = line[m.end(): anchors[i + 1].start() if i + 1 < len(anchors) else len(line)]
        lead = LEAD.match(seg)
        nums = [int(x) for x in re.findall(r"\d+", lead.group(0))] if lead else []
        rest = seg[lead.end():] if lead else seg
        for b in BARE.finditer(rest):
            nums += [int(x) for x in b.groups() if x]
        if nums:
            out.append((m.group(1), nums))
    return out


def test_continuation_parser():
    nw, bl, mn = "Networks" + ".py:", "Blocks" + ".py:", "main" + ".py:"   # split: not citations themselves
    assert cited_lines(nw + "35-37, 148-163 d") == [("Networks", [35, 37, 148, 163])]
    assert cited_lines("x " + nw + "29 / :170 (w)") == [("Networks", [29, 170])]
    assert cited_lines(nw + "27-33/:174-175 and the sum of :178 at") == [("Networks", [27, 33, 174, 175, 178])]
    assert cited_lines("(" + nw + "91, 184)") == [("Networks", [91, 184])]
    assert cited_lines(nw + "12-104 (shared, :107-108, :130-146)") == [("Networks", [12, 104, 107, 108, 130, 146])]
    assert cited_lines(mn + "92 and " + bl + "23, 63") == [("main", [92]), ("Blocks", [23, 63])]


def test_every_citation_is_in_range():
    lens = {n: len(_lines(n)) for n in FILES}
    bad = []
    for p in CITING:
        if not p.is_file() or p.suffix in (".o", ".so"):
            continue
        for k, line in enumerate(p.read_text(errors="replace").splitlines(), 1):
            for name, nums in cited_lines(line):
                if max(nums) > lens[name] + 1 or min(nums) < 1:
                    bad.append(f"{p.relative_to(ROOT)}:{k}: {name}.py {nums}")
    assert not bad, "citations past the end of the cited file:\n" + "\n".join(bad)


# (file, line) → text the line must contain: the anchors the product and the oracle cite most
ANCHORS = [
    ("Networks", 16, "def getModel"),
    ("Networks", 22, "name='objects'"),
    ("Networks", 29, "name='propagation'"),
    ("Networks", 32, "dot([permuted_senders_rel,objects]"),
    ("Networks", 46, "RelationalModel((n_relations,),2,[150,150,150,150])"),
    ("Networks", 50, "ObjectModel((n_objects,),300,[100,101])"),
    ("Networks", 75, "rel_encoding=Activation('relu')(rm("),
    ("Networks", 77, "Dropout(0.1)"),
    ("Networks", 83, "range(5)"),
    ("Networks", 86, "Concatenate()([rel_encoding,senders_prop,receivers_prop])"),
    ("Networks", 88, "dot([receiver_relations, x], axes=(2,1))"),
    ("Networks", 91, "Add()([prop_layer(x), prop])"),
    ("Networks", 94, "sigmoid(x[:,:,:1])"),
    ("Networks", 101, "optimizers.Adam(lr=0.0005"),
    ("Networks", 102, "binary_crossentropy"),
    ("Blocks", 23, "kernel_regularizer=regularizers.l2(regul)"),
    ("main", 78, "relation_threshold"),
    ("main", 92, "gnn_model.fit("),
    ("main", 96, "validation_split=0.2"),
]


@pytest.mark.parametrize("name,line,text", ANCHORS)
def test_anchor_lines(name, line, text):
    assert text in _lines(name)[line - 1]


def test_design_cites_the_mp_loop_and_loss():
    d = (ROOT / "DESIGN.md").read_text()
    assert "Networks.py:83" in d or "Networks.py:83-91" in d
    assert "Networks.py:77-78,101-102" in d
