"""Range-label stacks on the oracle: HierMergeBlock.rangeStacks rebuilt by blockUpdate
(addNodeReferences / applyStackDelta / applyRangeReference, mergeTree.ts:229-320, 2748-2767) and
MergeTree.getStackContext's search (rangeShift / recordRangeLeaf, mergeTree.ts:953-994, 1750-1760).

Pinned by the reference's own stack check (merge-tree/src/test/beastTest.ts:1403-1640,
DocumentTree.test1): a generated row / box / paragraph document inserted with NestBegin / NestEnd
markers (range labels "row" / "box", marker ids "row<n>" / "end-row<n>") gives, at every text
position, getStackContext(pos, ["box", "row"]) stacks whose marker ids equal the document's nesting
— the reference's checkStacksAllPositions.  The reference asserts nothing about stacks of labels
it did not ask for or about keys with empty stacks; those follow the restatement (block deltas
carry every label, an empty delta adds no key) and are compared GPU == oracle in
tests/test_gpu_writer.py (parity beyond this check is unpinned)."""
import random

import pytest

import oracle_ffi as O

TILE, NEST_BEGIN, NEST_END = 1, 2, 4


class DocTree:
    """beastTest.ts DocumentTree: Content -> (Row | Paragraph)*; Row -> row[Box*]; Box -> box[Content];
    Paragraph -> pg tile + text."""

    def __init__(self, name, children):
        self.name, self.children, self.id = name, children, None


def gen_content(rng, row_p):
    items = []
    for _ in range(rng.randint(7, 25)):
        if rng.randint(1, 1000) >= row_p * 1000:
            words = " ".join(rng.choice(["alpha", "beta", "gamma", "delta", "eps", "zeta"]) for _ in range(rng.randint(1, 6)))
            items.append(DocTree("pg", [words]))
        else:
            row_p /= 2
            if row_p < 0.08:
                row_p = 0
            items.append(DocTree("row", [DocTree("box", gen_content(rng, row_p)) for _ in range(rng.randint(1, 5))]))
    return items


def add_to_tree(d, node, st):
    """addToMergeTree (beastTest.ts:1414-1462) as local ops of the collaborating client"""
    if isinstance(node, str):
        assert d.local_op({"type": 0, "pos1": st["pos"], "seg": node}) == 0, d.error
        st["pos"] += len(node)
        return
    if node.name == "pg":
        seg = {"marker": {"refType": TILE}, "props": {"referenceTileLabels": ["pg"]}}
        assert d.local_op({"type": 0, "pos1": st["pos"], "seg": seg}) == 0
        st["pos"] += 1
    else:
        node.id = f"{node.name}{st['ids'][node.name]}"
        st["ids"][node.name] += 1
        props = {"markerId": node.id, "referenceRangeLabels": [node.name]}
        behaviors = NEST_BEGIN
        if node.name == "row":
            props["referenceTileLabels"] = ["pg"]
            behaviors |= TILE
        assert d.local_op({"type": 0, "pos1": st["pos"], "seg": {"marker": {"refType": behaviors}, "props": props}}) == 0
        st["pos"] += 1
    for c in node.children:
        add_to_tree(d, c, st)
    if node.name != "pg":
        props = {"markerId": f"end-{node.id}", "referenceRangeLabels": [node.name]}
        assert d.local_op({"type": 0, "pos1": st["pos"], "seg": {"marker": {"refType": NEST_END}, "props": props}}) == 0
        st["pos"] += 1


def check_stacks_all_positions(d, children):
    """checkStacksAllPositions (beastTest.ts:1464-1540): at every text node, the client's stacks for
    "box" / "row" hold exactly the enclosing begin markers' ids, outermost first"""
    errors = []
    model = {"box": [], "row": []}
    pos = 0

    def walk(node):
        nonlocal pos
        if isinstance(node, str):
            got = d.stack_context(pos, ["box", "row"])
            for name in ("box", "row"):
                ids = [it.get("props", {}).get("markerId") for it in got.get(name, [])]
                if ids != model[name]:
                    errors.append((pos, name, ids, list(model[name])))
            pos += len(node)
            return
        pos += 1
        if node.name == "pg":
            walk(node.children[0])
            return
        model[node.name].append(node.id)
        for c in node.children:
            walk(c)
        model[node.name].pop()
        pos += 1

    for c in children:
        walk(c)
    return errors


@pytest.mark.parametrize("seed", range(6))
def test_document_tree_stacks_at_every_position(seed):
    """DocumentTree.test1 (beastTest.ts:1580-1584) on generated documents: 0 errors"""
    rng = random.Random(seed)
    children = gen_content(rng, 0.6)
    d = O.Doc()
    d.start_collab("Fred")
    st = {"pos": 0, "ids": {"box": 0, "row": 0}}
    for c in children:
        add_to_tree(d, c, st)
    assert d.length() == st["pos"]
    assert check_stacks_all_positions(d, children) == []


def test_stack_context_quirks():
    """The restatement's reading of the search: a preceding block contributes its whole delta (every
    label, including ones not asked for); preceding leaves of the containing leaf block and the
    containing leaf contribute only the asked-for labels; a delta that reduces to an empty stack adds
    no key; an end marker pops any begin on top (labels are not matched)."""
    d = O.Doc()
    d.start_collab("Fred")
    mk = lambda rt, lab, mid: {"marker": {"refType": rt}, "props": {"markerId": mid, "referenceRangeLabels": lab}}
    segs = [mk(NEST_BEGIN, ["a"], "a0"), "xx", mk(NEST_BEGIN, ["b"], "b0"), "yy", mk(NEST_END, ["b"], "b0e"),
            mk(NEST_BEGIN, ["a", "b"], "ab1"), "zz"] + ["t%d" % i for i in range(20)]
    pos = 0
    for s in segs:
        assert d.local_op({"type": 0, "pos1": pos, "seg": s}) == 0
        pos += 1 if isinstance(s, dict) else len(s)
    end = d.length()
    only_a = d.stack_context(end - 1, ["a"])  # deep in the trailing text: the markers lie in preceding blocks
    assert [it["props"]["markerId"] for it in only_a["a"]] == ["a0", "ab1"]
    assert [it["props"]["markerId"] for it in only_a.get("b", [])] == ["ab1"]  # not asked for, but in a block delta
    first = d.stack_context(0, ["a"])  # the containing leaf is the first begin marker
    assert [it["props"]["markerId"] for it in first["a"]] == ["a0"]
    assert list(first) == ["a"]
