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
    *ROOT.glob("include/*.h"), ROOT / "DESIGN.md", ROOT / "INTEGRATION.md", ROOT / "README.md",
    ROOT / "bench.py", *ROOT.glob("tests/*.py"),
]
PAT = re.compile(r"\b(Networks|Blocks|main|JengaBuilder|TowerCreator)\.py:(\d+(?:[-,]\d+)*)")


def _lines(name):
    return (REF / f"{name}.py").read_text().splitlines()


def test_every_citation_is_in_range():
    lens = {n: len(_lines(n)) for n in ("Networks", "Blocks", "main", "JengaBuilder", "TowerCreator")}
    bad = []
    for p in CITING:
        if not p.is_file() or p.suffix in (".o", ".so"):
            continue
        for m in PAT.finditer(p.read_text(errors="replace")):
            nums = [int(x) for x in re.findall(r"\d+", m.group(2))]
            if max(nums) > lens[m.group(1)] + 1 or min(nums) < 1:
                bad.append(f"{p.relative_to(ROOT)}: {m.group(0)}")
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
