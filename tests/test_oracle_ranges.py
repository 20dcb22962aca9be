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


# Derived known-answer cases for getStackContext.  Nothing in the reference's tests pins these
# values: they are worked by hand from the reference's rules and are marked "derived".
#   applyRangeReference (mergeTree.ts:246-261): a NestBegin pushes; an end pops a NestBegin on top
#     and is pushed otherwise (no label matching beyond the per-label stack).
#   applyLeafRangeMarker (953-964): a leaf marker touches only the requested labels, in request
#     order, creating a label's stack on first touch (it may end empty).
#   applyStackDelta (229-244) via rangeShift (978-994): a preceding block applies its whole
#     rangeStacks delta, every label, skipping labels whose delta stack is empty.
#   split (2476-2489) at MaxNodesInBlock 8: appending segments one by one leaves segments 0..3 in
#     the first leaf block for good once the 8th is inserted, so with >= 8 segments a query past
#     segment 3 sees segments 0..3 only through that block's delta.
# The output shape {label: [{pos, refType, props}, ...]} (stacks bottom to top, labels in the
# order the search created them) is this repo's rendering of searchInfo.stacks, not the
# reference's (a RangeStackMap of Stack<Marker>): INTEGRATION.md.
def _mk(rt, labels, mid):
    return {"marker": {"refType": rt}, "props": {"markerId": mid, "referenceRangeLabels": labels}}


def _it(pos, rt, labels, mid):
    return {"pos": pos, "refType": rt, "props": {"markerId": mid, "referenceRangeLabels": labels}}


_E0, _AB, _EB = (NEST_END, ["a"], "e0"), (NEST_BEGIN, ["a", "b"], "ab"), (NEST_END, ["b"], "eb")
_A0, _B0, _B0E, _C0E = (NEST_BEGIN, ["a"], "a0"), (NEST_BEGIN, ["b"], "b0"), (NEST_END, ["b"], "b0e"), (NEST_END, ["c"], "c0e")
_AE = (NEST_END, ["a"], "ae")
STACK_KATS = [
    {   # one leaf block: every marker is a leaf the search visits, so only requested labels count
        "name": "single_block",
        "segs": [_mk(*_E0), _mk(*_AB), "xx", _mk(*_EB), "yy"],
        "queries": [
            (5, ["a", "b"], {"a": [_it(0, *_E0), _it(1, *_AB)], "b": []}),  # end on an empty stack is pushed; eb pops ab
            (5, ["b"], {"b": []}),                                            # e0 has no "b": no "a" key
            (0, ["a"], {"a": [_it(0, *_E0)]}),                                # the containing leaf applies too
            (1, ["b", "a"], {"a": [_it(0, *_E0), _it(1, *_AB)], "b": [_it(1, *_AB)]}),  # keys in creation order
            (2, ["a", "b"], {"a": [_it(0, *_E0), _it(1, *_AB)], "b": [_it(1, *_AB)]}),
            (4, ["b"], {"b": []}),                                            # containing end pops the begin below
            (6, [], {}),
        ],
    },
    {   # markers in the first leaf block, queried from later blocks: the block delta carries every label
        "name": "block_delta",
        "segs": [_mk(*_A0), _mk(*_B0), _mk(*_B0E), _mk(*_C0E)] + ["t%02d" % i for i in range(20)],
        "queries": [
            (63, ["a"], {"a": [_it(0, *_A0)], "c": [_it(3, *_C0E)]}),  # "b" delta is empty: skipped
            (4, [], {"a": [_it(0, *_A0)], "c": [_it(3, *_C0E)]}),
            (3, ["a"], {"a": [_it(0, *_A0)]}),                          # same block: leaves, requested labels only
            (3, ["b"], {"b": []}),
            (3, ["c"], {"c": [_it(3, *_C0E)]}),
        ],
    },
    {   # a begin in block 0 popped by the end in block 1's delta: the key stays with an empty stack
        "name": "pop_across_blocks",
        "segs": [_mk(*_A0), "t0", "t1", "t2", _mk(*_AE)] + ["u%02d" % i for i in range(16)],
        "queries": [
            (60, [], {"a": []}),
            (4, ["a"], {"a": [_it(0, *_A0)]}),                          # in "t1": leaves of block 0
            (7, ["a"], {"a": []}),                                      # on ae itself: block 0 delta, then ae pops
            (8, ["b"], {"a": [_it(0, *_A0)]}),                          # ae is a leaf of this block, "a" not asked for
            (20, ["b"], {"a": []}),                                     # past block 1: both block deltas
        ],
    },
]


def stack_kat_messages(kat, client="W"):
    """The KAT's segments as one writer's sequenced inserts, appended in order; minimumSequenceNumber
    stays 0 so no zamboni merges segments and the block shape is the append shape."""
    msgs, pos = [], 0
    for i, s in enumerate(kat["segs"]):
        msgs.append({"clientId": client, "sequenceNumber": i + 1, "referenceSequenceNumber": i,
                     "minimumSequenceNumber": 0, "type": "op", "contents": {"type": 0, "pos1": pos, "seg": s}})
        pos += 1 if isinstance(s, dict) else len(s)
    return msgs


@pytest.mark.parametrize("kat", STACK_KATS, ids=lambda k: k["name"])
def test_stack_context_derived_kats(kat):
    """derived (hand-worked, not reference fixtures): the writer's local view and a read-only
    replica of its sequenced ops both give the worked stacks"""
    import json

    w = O.Doc()
    w.start_collab("W")
    obs = O.Doc()
    obs.start_collab("readonly")
    for m in stack_kat_messages(kat):
        assert w.local_op(m["contents"]) == 0, w.error
        assert obs.apply_msg(json.dumps(m)) == 0, obs.error
    for d in (w, obs):
        for pos, labels, want in kat["queries"]:
            got = d.stack_context(pos, labels)
            assert got == want, (kat["name"], pos, labels, got)
            assert list(got) == list(want), (kat["name"], pos, labels)
