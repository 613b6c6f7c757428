"""Golden vectors (tests/golden/*.json, made by tests/golden/make_golden.py).

CPU: the oracle still reproduces every vector; the host codec round-trips every state.
GPU: the lasp_orset / lasp_gset / lasp_lattice mirrors, running on the device through
the C ABI, reproduce every vector bit for bit (tokens and flags included).
"""

import json
import os

import numpy as np
import pytest

from oracle import core, gset, lattice, orset
from tests.golden.termjson import dec

HERE = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def _load(name):
    with open(os.path.join(HERE, name)) as f:
        return json.load(f)["cases"]


OR = _load("orset_cases.json")
GS = _load("gset_cases.json")


def _eq(a, b):
    from oracle.terms import exact_eq
    return exact_eq(a, b)


# ------------------------------------------------------------------ CPU: oracle pin

def test_oracle_reproduces_orset_vectors():
    for c in OR:
        a, b = dec(c["a"]), dec(c["b"])
        assert _eq(orset.merge(a, b), dec(c["merge"]))
        assert _eq(orset.value(a), dec(c["value_a"]))
        assert lattice.is_inflation("lasp_orset", a, dec(c["merge"])) is c["infl_a_m"]
        assert _eq(core.intersection_body("lasp_orset", a, b), dec(c["intersection"]))


def test_oracle_reproduces_gset_vectors():
    for c in GS:
        a, b = dec(c["a"]), dec(c["b"])
        assert _eq(gset.merge(a, b), dec(c["merge"]))
        assert lattice.is_strict_inflation("lasp_gset", a, dec(c["merge"])) is c["strict_a_m"]


def test_vectors_cover_edge_cases():
    assert any(dec(c["a"]) == [] for c in OR)                       # empty
    assert any(c["equal_ab"] for c in OR)                           # identical
    assert any(dec(c["removed_a"]) for c in OR)                     # tombstones
    assert any(not c["infl_b_a"] for c in OR)                       # non-inflations
    assert any(c["map_x2"] is None for c in OR)                     # mixed-term sets


# ------------------------------------------------------------------ CPU: host codec

def test_codec_roundtrip_orset():
    from lasp_amd.codec import Domain
    from lasp_amd.terms import Atom
    for c in OR:
        a = dec(c["a"], Atom)
        m = dec(c["merge"], Atom)
        dom = Domain()
        dom.register_orset(a)
        dom.register_orset(m)
        cells = dom.encode_orset([a, m], max(1, dom.size))
        assert _eq(dom.decode_orset(cells[0]), a)
        assert _eq(dom.decode_orset(cells[1]), m)


def test_codec_rejects_noncanonical():
    from lasp_amd.codec import Domain, NonCanonical
    dom = Domain()
    with pytest.raises(NonCanonical):
        dom.encode_orset([[(2, [(b"t", False)]), (1, [(b"t", False)])]], 4)   # unsorted
    with pytest.raises(NonCanonical):
        dom.encode_orset([[(1, [(b"t", False)]), (1, [(b"u", False)])]], 4)   # duplicate
    with pytest.raises(NonCanonical):
        dom.encode_orset([[(1, [])]], 4)                                       # no tokens
    with pytest.raises(NonCanonical):
        dom.encode_gset([[1, 2, 3, 2, 3, 4]], 8)          # G-Set union L ++ R output


def test_codec_capacity():
    from lasp_amd.codec import CapacityError, Domain
    dom = Domain()
    s = [(1, [(bytes([k]) * 20, False) for k in range(65)])]
    with pytest.raises(CapacityError):
        dom.encode_orset([s], 4)


# ------------------------------------------------------------------ GPU: mirrors

@pytest.mark.gpu
def test_gpu_orset_mirror_matches_vectors():
    from lasp_amd import lattice as dl
    from lasp_amd import orset as do
    from lasp_amd.terms import Atom
    pairs = [(dec(c["a"], Atom), dec(c["b"], Atom)) for c in OR]
    merged = do.merge_many(pairs)                     # one launch for all 60 pairs
    for c, (a, b), m in zip(OR, pairs, merged):
        assert _eq(m, dec(c["merge"]))
        assert _eq(do.merge(a, b), dec(c["merge"]))
        assert _eq(do.value(a), dec(c["value_a"]))
        assert _eq(do.value2("removed", a), dec(c["removed_a"]))
        assert [list(x) for x in do.stats(a)] == c["stats_a"]
        assert do.equal(a, b) is c["equal_ab"]
        mm = dec(c["merge"], Atom)
        assert dl.is_inflation("lasp_orset", a, mm) is c["infl_a_m"]
        assert dl.is_inflation("lasp_orset", b, a) is c["infl_b_a"]
        assert dl.is_strict_inflation("lasp_orset", a, mm) is c["strict_a_m"]
        assert dl.is_strict_inflation("lasp_orset", a, a) is c["strict_a_a"]
        assert dl.is_strict_inflation("lasp_orset", b, a) is c["strict_b_a"]
        assert dl.threshold_met("lasp_orset", mm, ("strict", a)) is c["strict_a_m"]


@pytest.mark.gpu
def test_gpu_orset_union_filter_match_vectors():
    from lasp_amd import orset as do
    from lasp_amd.codec import Domain
    from lasp_amd.terms import Atom
    ctx = do.context()
    for c in OR:
        a, b = dec(c["a"], Atom), dec(c["b"], Atom)
        dom = Domain()
        dom.register_orset(a)
        dom.register_orset(b)
        E = max(1, dom.size)
        L, R, U, F = (ctx.orset_batch(1, E) for _ in range(4))
        L.upload(dom.encode_orset([a], E))
        R.upload(dom.encode_orset([b], E))
        U.union(L, R)
        F.filter(L, dom.keep_bits(lambda x: isinstance(x, int) and x % 2 == 0, E))
        assert _eq(dom.decode_orset(U.download()[0]), dec(c["union"]))
        assert _eq(dom.decode_orset(F.download()[0]), dec(c["filter_even"]))


@pytest.mark.gpu
def test_gpu_gset_mirror_matches_vectors():
    from lasp_amd import gset as dg
    from lasp_amd import lattice as dl
    from lasp_amd.terms import Atom
    for c in GS:
        a, b = dec(c["a"], Atom), dec(c["b"], Atom)
        m = dec(c["merge"], Atom)
        assert _eq(dg.merge(a, b), dec(c["merge"]))
        assert dg.equal(a, b) is c["equal_ab"]
        assert dl.is_inflation("lasp_gset", a, m) is c["infl_a_m"]
        assert dl.is_inflation("lasp_gset", b, a) is c["infl_b_a"]
        assert dl.is_strict_inflation("lasp_gset", a, m) is c["strict_a_m"]
        assert dl.is_strict_inflation("lasp_gset", m, m) is c["strict_m_m"]
        assert [list(x) for x in dg.stats(a)] == c["stats_a"]


@pytest.mark.gpu
def test_gpu_orset_update_matches_oracle():
    """update/3 sequences on the device vs the oracle (add_by_token / remove / errors)."""
    from lasp_amd import orset as do
    from lasp_amd.terms import Atom
    toks = [bytes([k + 1]) * 20 for k in range(10)]
    ops = [("add_by_token", toks[0], 1), ("add_by_token", toks[1], 1), ("remove", 1),
           ("add_by_token", toks[2], Atom("x")), ("remove", 5),
           ("update", [("add_by_token", toks[3], 2), ("remove", 9)]),
           ("update", [("add_by_token", toks[4], 3), ("remove", 3)]),
           ("remove_all", [1, Atom("x")]), ("remove_all", [1, 77]),
           ("add_by_token", toks[0], 1)]
    so, sd = orset.new(), do.new()
    for op in ops:
        ro = orset.update(op, None, so)
        rd = do.update(op, None, sd)
        assert ro[0] == rd[0], op
        if ro[0] == "ok":
            so, sd = ro[1], rd[1]
            assert _eq(sd, so), op
        else:
            assert _eq(rd[1], ro[1]), op
    st = do.stats(sd)
    assert [list(x) for x in st] == [list(x) for x in orset.stats(so)]
    np.testing.assert_equal(len(do.value(sd)), len(orset.value(so)))


@pytest.mark.gpu
def test_gpu_orset_combinator_bodies_match_vectors():
    """intersection / product / map / fold bodies (lasp_core.erl:460-667) on the device,
    decoded list-faithfully (Cx ++ Cy, descending product tokens, duplicates kept)."""
    from lasp_amd import orset as do
    from lasp_amd.codec import Domain, SeqOutput, decode_concat, decode_product
    from lasp_amd.terms import Atom
    ctx = do.context()
    for c in OR:
        a, b = dec(c["a"], Atom), dec(c["b"], Atom)
        dom = Domain()
        dom.register_orset(a)
        dom.register_orset(b)
        E = max(1, dom.size)
        L, R = ctx.orset_batch(1, E), ctx.orset_batch(1, E)
        L.upload(dom.encode_orset([a], E))
        R.upload(dom.encode_orset([b], E))
        X = L.intersection(R)
        assert _eq(decode_concat(dom, X.download()[0]), dec(c["intersection"]))
        # product of the first 4 elements of each side, each in its own domain
        dl, dr = Domain(), Domain()
        dl.register_orset(a[:4])
        dr.register_orset(b[:4])
        PL, PR = ctx.orset_batch(1, max(1, dl.size)), ctx.orset_batch(1, max(1, dr.size))
        PL.upload(dl.encode_orset([a[:4]], PL.elements))
        PR.upload(dr.encode_orset([b[:4]], PR.elements))
        P = PL.product(PR)
        assert _eq(decode_product(dl, dr, P.download()[0]), dec(c["product"]))
        # fold X -> [X, X, X] and map X -> 2X over the dictionary, gathered on device
        fo = SeqOutput.fold(dom, lambda x: [x, x, x])
        F = ctx.orset_batch(1, max(1, fo.size)).gather(L, fo.index())
        assert _eq(fo.decode_orset(F.download()[0]), dec(c["fold_x3"]))
        if c["map_x2"] is not None:
            mo = SeqOutput.map(dom, lambda x: x * 2)
            M = ctx.orset_batch(1, max(1, mo.size)).gather(L, mo.index())
            assert _eq(mo.decode_orset(M.download()[0]), dec(c["map_x2"]))
