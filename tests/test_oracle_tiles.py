"""findTile on the oracle (block tile maps rebuilt by blockUpdate, search / backwardSearch:
mergeTree.ts:263-318, 998-1035, 1763-1874), pinned by the reference's client.spec.ts KATs; and the
final-table scan the library uses (mt_doc_find_tile) restated here and checked against the maps on
random documents with markers."""
import json

import pytest

import oracle_ffi as O
from writer_sim import TILE_LABELS, farm, round_farm

EOP = "EOP"


def marker(label=EOP, ref_type=1):
    return {"marker": {"refType": ref_type}, "props": {"referenceTileLabels": [label], "markerId": "some-id"}}


@pytest.fixture
def client():
    """client.spec.ts:16-26: a collaborating client (its beforeEach's empty segment inserts nothing)."""
    d = O.Doc()
    d.start_collab("localUser")
    return d


def ins(d, pos, seg):
    assert d.local_op({"type": 0, "pos1": pos, "seg": seg}) == 0


def test_non_preceding_tile(client):  # :29-51
    ins(client, 0, marker())
    ins(client, 0, "abc")
    assert client.length() == 4
    assert client.find_tile(0, EOP, False)["pos"] == 3


def test_non_preceding_single_tile(client):  # :53-73
    ins(client, 0, "abc d")
    ins(client, 0, marker())
    assert client.length() == 6
    assert client.find_tile(0, EOP, False)["pos"] == 0


def _three_tiles(client):  # :75-102 / :114-141
    ins(client, 0, marker())
    ins(client, 0, "abc d")
    ins(client, 0, marker())
    ins(client, 7, "ef")
    ins(client, 8, marker())
    assert client.length() == 10


def test_preceding_tile_of_several(client):  # :75-112
    _three_tiles(client)
    assert client.find_tile(5, EOP)["pos"] == 0


def test_non_preceding_tile_of_several(client):  # :114-151
    _three_tiles(client)
    assert client.find_tile(5, EOP, False)["pos"] == 6


def test_tile_in_a_length_1_text(client):  # :153-179
    ins(client, 0, marker())
    assert client.length() == 1
    assert client.find_tile(0, EOP)["pos"] == 0
    assert client.find_tile(0, EOP, False)["pos"] == 0


def test_index_out_of_bound(client):  # :181-205
    ins(client, 0, marker())
    ins(client, 0, "abc")
    assert client.find_tile(5, EOP)["pos"] == 3
    assert client.find_tile(5, EOP, False) is None


def test_text_without_the_tile(client):  # :207-219
    ins(client, 0, "abc")
    assert client.find_tile(1, EOP) is None
    assert client.find_tile(1, EOP, False) is None


def test_null_text(client):  # :221-231
    assert client.find_tile(1, EOP) is None
    assert client.find_tile(1, EOP, False) is None


def leaf_list(d, label):
    leaves = []
    for ln in d.dump().splitlines():
        ln = ln.strip()
        if not ln.startswith("S "):
            continue
        n = int(ln.split("len=")[1].split()[0])
        removed = ln.split("rseq=")[1].split()[0] != "none"
        lab = None
        if " rt=" in ln and int(ln.split(" rt=")[1].split()[0]) & 1:
            props = json.loads(ln[ln.rindex("' ") + 2:]) if ln.rstrip().endswith("}") else {}
            lab = props.get("referenceTileLabels")
        leaves.append((0 if removed else n, lab is not None and label in lab))
    return leaves


def scan_find_tile(leaves, start_pos, preceding=True):
    """mt_doc_find_tile's rule over the final leaf list (local view)."""
    total = sum(n for n, _ in leaves)
    pos, k = 0, 0
    while k < len(leaves) and not start_pos < pos + leaves[k][0]:
        pos += leaves[k][0]
        k += 1
    found = None
    if preceding:
        if k < len(leaves) and leaves[k][1]:
            found = k
        else:
            for i in range(min(k, len(leaves)) - 1, -1, -1):
                if leaves[i][0] > 0 and leaves[i][1]:
                    found = i
                    break
    elif start_pos < total:
        found = k if leaves[k][1] else next((i for i in range(k + 1, len(leaves)) if leaves[i][0] > 0 and leaves[i][1]), None)
    elif start_pos == total and leaves and leaves[-1][1]:
        found = len(leaves) - 1
    return None if found is None else sum(n for n, _ in leaves[:found])


@pytest.mark.parametrize("mk", [lambda: round_farm(4, 30, 31, markers=30), lambda: farm(5, 600, 32, markers=25)])
def test_block_tile_maps_equal_the_final_table_scan(mk):
    """The reference's map-based search == the scan over the final table, on every replica of
    farms with Tile markers (inserted, removed, split around, packed by zamboni)."""
    f = mk()
    replicas = list(f.docs.values()) + [f.observer]
    checked = 0
    for d in replicas:
        n = d.length()
        for label in TILE_LABELS:
            leaves = leaf_list(d, label)
            for pos in range(0, n + 2):
                for prec in (True, False):
                    got = d.find_tile(pos, label, prec)
                    assert (None if got is None else got["pos"]) == scan_find_tile(leaves, pos, prec), (pos, label, prec)
                    checked += got is not None
    assert checked > 100
