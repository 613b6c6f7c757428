"""The native host side of the boundary (laspj_term_compare, laspj_dict_*), on the CPU:
the term-order comparator against the Python restatement of Erlang term order
(lasp_amd.terms.term_cmp, which the oracle's KATs rely on), and the dictionary + encoder
against the Python codec (codec.Domain) on random orddicts / ordsets written as
term_to_binary/1 payloads (lasp_amd.etf)."""

import ctypes as C
import struct

import numpy as np
import pytest
from hypothesis import HealthCheck, given, settings, strategies as st

from lasp_amd import _lib, etf
from lasp_amd.codec import Domain
from lasp_amd.terms import Atom, term_cmp

SOAK = int(__import__("os").environ.get("LASPJ_SOAK", "1"))   # x examples for a soak run

ATOMS = st.sampled_from([Atom(a) for a in ("a", "b", "abc", "zz", "é", "ünïcode", "true", "false")])
NUM = st.one_of(st.integers(-(1 << 70), 1 << 70), st.integers(-300, 300),
                st.floats(allow_nan=False, allow_infinity=False, width=64),
                st.sampled_from([0, 1, 1.0, -1, 255, 256, 2 ** 31, 2 ** 63, 0.5, -0.0]))
LEAF = st.one_of(NUM, ATOMS, st.binary(max_size=6), st.just([]),
                 st.lists(st.integers(0, 255), max_size=4))
TERM = st.recursive(LEAF, lambda ch: st.one_of(st.tuples(ch, ch), st.tuples(ch),
                                               st.lists(ch, max_size=3)), max_leaves=6)


@pytest.fixture(scope="module")
def lib():
    from lasp_amd import build
    build.build()
    return _lib.load()


def compare(lib, a, b):
    x, y = etf.encode(a), etf.encode(b)
    out = C.c_int()
    st_ = lib.laspj_term_compare(x, len(x), y, len(y), C.byref(out))
    assert st_ == 0, (a, b)
    return out.value


@settings(max_examples=600 * SOAK, deadline=None, suppress_health_check=[HealthCheck.too_slow])
@given(TERM, TERM)
def test_term_compare_matches_erlang_order(lib, a, b):
    assert compare(lib, a, b) == term_cmp(a, b), (a, b)
    assert compare(lib, a, a) == 0


def test_term_compare_edges(lib):
    assert compare(lib, 1, 1.0) == 0                  # numbers compare by value
    assert compare(lib, 2 ** 64 + 1, 1.8446744073709552e19) == 1
    assert compare(lib, -(2 ** 70), -1e21) == -1
    assert compare(lib, [1, 2], [1, 2, 0]) == -1      # STRING_EXT vs STRING_EXT prefix
    assert compare(lib, [1, 2], [1, Atom("a")]) == -1  # STRING_EXT vs LIST_EXT
    assert compare(lib, (1,), [1]) == -1               # tuple < list
    assert compare(lib, [], [0]) == -1                 # nil < list
    assert compare(lib, b"", []) == 1                  # bitstring > everything
    out = C.c_int()
    bad = bytes([116, 0, 0, 0, 0])                     # a map: outside this path
    assert lib.laspj_term_compare(bad, 5, bad, 5, C.byref(out)) == _lib.E_UNSUPPORTED


class NDict:
    """the test's view: lasp_amd.hostdict.NativeDict with the library fixture"""

    def __init__(self, lib):
        from lasp_amd.hostdict import NativeDict
        self.n = NativeDict()
        self.h = self.n.h

    def add(self, kind, payloads, tag=-1):
        return self.n.add(kind, payloads, tag)

    def export(self, E, tokens=True):
        return self.n.export(E, tokens)

    def encode(self, kind, payloads, E, tag=-1):
        return self.n.encode(kind, payloads, E, tag)


def orsets(draw_ops, seed):
    from oracle import orset
    toks = orset.TokenSource(seed)
    s = orset.new()
    for kind, e in draw_ops:
        op = ("add_by_token", toks(), e) if kind == "add" else ("remove", e)
        r = orset.update(op, None, s)
        if r[0] == "ok":
            s = r[1]
    return s


ELEMS = st.one_of(st.integers(-5, 300), ATOMS, st.tuples(st.integers(0, 3), ATOMS),
                  st.binary(min_size=1, max_size=3))
OPS = st.lists(st.tuples(st.sampled_from(["add", "add", "remove"]), ELEMS), max_size=20)


@settings(max_examples=120 * SOAK, deadline=None, suppress_health_check=[HealthCheck.too_slow])
@given(st.lists(OPS, min_size=1, max_size=4))
def test_dict_export_and_encode_match_python_codec(lib, opss):
    values = [orsets(ops, 10 + i) for i, ops in enumerate(opss)]
    payloads = [bytes([76, 1]) + etf.term_to_binary(v) for v in values]
    d = NDict(lib)
    assert list(d.add(_lib.KIND_ORSET, payloads, tag=76)) == [0] * len(values)
    dom = Domain()
    for v in values:
        dom.register_orset(v)
    E = max(1, dom.size) + 3
    eb, eo, eord, tb, to, tord = d.export(E)
    peb, peo, peord, ptb, pto, ptord = dom.etf_arrays(E)
    # slots are assigned in first-seen order by both: images and orders must agree
    assert eb == peb and np.array_equal(eo, peo) and np.array_equal(eord, peord)
    assert tb == ptb and np.array_equal(to, pto) and np.array_equal(tord, ptord)
    cells, st_ = d.encode(_lib.KIND_ORSET, payloads, E, tag=76)
    assert list(st_) == [0] * len(values)
    want = dom.encode_orset(values, E).reshape(len(values), 2 * E)
    assert np.array_equal(cells, want)


@settings(max_examples=80 * SOAK, deadline=None)
@given(st.lists(st.lists(ELEMS, max_size=12), min_size=1, max_size=4))
def test_gset_dict_and_encode(lib, sets):
    from oracle import otp
    values = [otp.lists_usort(s) for s in sets]
    payloads = [etf.term_to_binary(v) for v in values]
    d = NDict(lib)
    assert list(d.add(_lib.KIND_GSET, payloads)) == [0] * len(values)
    dom = Domain()
    E = 1
    gw = dom.encode_gset(values, 4096)
    E = max(1, dom.size)
    eb, eo, eord, *_ = d.export(E, tokens=False)
    peb, peo, peord, *_ = dom.etf_arrays(E, tokens=False)
    assert eb == peb and np.array_equal(eord, peord)
    words, st_ = d.encode(_lib.KIND_GSET, payloads, E)
    assert list(st_) == [0] * len(values)
    W = (E + 63) // 64
    assert np.array_equal(words, gw[:, :W])


def test_dict_statuses(lib):
    d = NDict(lib)
    tok = b"t" * 20
    good = etf.term_to_binary([(1, [(tok, False)]), (2, [(tok, True)])])
    unsorted = etf.term_to_binary([(2, [(tok, False)]), (1, [(tok, False)])])
    dup_tok = etf.term_to_binary([(1, [(tok, False), (tok, True)])])
    no_toks = etf.term_to_binary([(1, [])])
    bad_flag = etf.term_to_binary([(1, [(tok, Atom("maybe"))])])
    truncated = good[:-3]
    st_ = d.add(_lib.KIND_ORSET, [good, unsorted, dup_tok, no_toks, bad_flag, truncated,
                                  bytes([76, 2]) + good[0:0] + good])
    assert list(st_) == [_lib.DEC_OK, _lib.DEC_OK, _lib.DEC_OK, _lib.DEC_UNREPRESENTABLE,
                         _lib.DEC_MALFORMED, _lib.DEC_MALFORMED, _lib.DEC_MALFORMED]
    assert list(d.add(_lib.KIND_ORSET, [bytes([76, 2]) + good, bytes([9, 1]) + good],
                      tag=76)) == [_lib.DEC_OK, _lib.DEC_INVALID_BINARY]
    cells, st_ = d.encode(_lib.KIND_ORSET, [good, unsorted, dup_tok], 4)
    # not an orddict (keys / tokens not strictly ascending): the list path takes it
    assert list(st_) == [_lib.DEC_OK, _lib.DEC_UNKNOWN_TERM, _lib.DEC_UNKNOWN_TERM]
    assert not cells[1].any() and not cells[2].any()
    many = etf.term_to_binary([(7, [(bytes([k]) * 20, False) for k in range(65)])])
    assert list(d.add(_lib.KIND_ORSET, [many])) == [_lib.DEC_UNREPRESENTABLE]
    st2 = np.zeros((1,), np.int32)
    assert lib.laspj_dict_add(d.h, _lib.KIND_GCOUNTER, good, np.array([0, len(good)],
                              np.uint64).ctypes.data, 1, -1, st2.ctypes.data) == _lib.E_KIND


def test_dict_encode_rejects_descending_offsets(lib):
    """laspj_dict_encode checks offsets like laspj_dict_add: a descending pair is
    LASPJ_E_INVAL, never a read past the blob."""
    from lasp_amd.hostdict import NativeDict
    d = NativeDict()
    p = etf.term_to_binary([(1, [(b"t" * 20, False)])])
    assert list(d.add(_lib.KIND_ORSET, [p])) == [_lib.DEC_OK]
    blob = C.create_string_buffer(p, len(p))
    offs = np.array([len(p), 0], np.uint64)            # offsets[1] < offsets[0]
    out = np.zeros((1, 2), np.uint64)
    st_ = np.zeros((1,), np.int32)
    assert lib.laspj_dict_encode(d.h, _lib.KIND_ORSET, blob, offs.ctypes.data, 1, -1, 1,
                                 out.ctypes.data, st_.ctypes.data) == _lib.E_INVAL
    with pytest.raises(_lib.LaspjError):
        lib_add = lib.laspj_dict_add(d.h, _lib.KIND_ORSET, blob, offs.ctypes.data, 1, -1,
                                     st_.ctypes.data)
        _lib.check(lib_add)


def test_dict_add_failed_payload_registers_nothing(lib):
    """A payload that fails (truncated, or an element past 64 tokens) leaves the
    dictionary exactly as it was: binary_to_term/1 rejects the whole payload, so none of
    its terms may take an element or token slot."""
    from lasp_amd.hostdict import NativeDict
    d = NativeDict()
    good = etf.term_to_binary([(1, [(b"a" * 20, False)]), (2, [(b"b" * 20, True)])])
    assert list(d.add(_lib.KIND_ORSET, [good])) == [_lib.DEC_OK]
    before = d.info()
    exp_before = d.export(4)
    # new elements 3, 4 and a new token of 1, then the payload is cut short
    bad = etf.term_to_binary([(1, [(b"a" * 20, False), (b"c" * 20, False)]),
                              (3, [(b"d" * 20, False)]), (4, [(b"e" * 20, False)])])
    for cut in (len(bad) - 1, len(bad) - 9, len(bad) // 2):
        st_ = d.add(_lib.KIND_ORSET, [bad[:cut]])
        assert st_[0] == _lib.DEC_MALFORMED
        assert d.info() == before
    # 65 distinct tokens for one new element: UNREPRESENTABLE, nothing kept
    many = etf.term_to_binary([(9, [(bytes([k]) * 20, False) for k in range(65)])])
    assert d.add(_lib.KIND_ORSET, [many])[0] == _lib.DEC_UNREPRESENTABLE
    assert d.info() == before
    exp_after = d.export(4)
    for x, y in zip(exp_before, exp_after):
        assert (x == y) if isinstance(x, bytes) else np.array_equal(x, y)
    # the same terms register normally once the payload is whole, in first-seen order
    assert d.add(_lib.KIND_ORSET, [bad])[0] == _lib.DEC_OK
    assert d.info()[0] == 4
    cells, st2 = d.encode(_lib.KIND_ORSET, [bad], 4)
    assert st2[0] == _lib.DEC_OK
    assert int(cells[0, 0]) == 0b11 and int(cells[0, 4]) == 1 and int(cells[0, 6]) == 1
    # G-Set payloads too
    g = etf.term_to_binary([100, 200, 300])
    assert d.add(_lib.KIND_GSET, [g[:-2]])[0] == _lib.DEC_MALFORMED
    assert d.info()[0] == 4


def test_domain_journal_undoes_failed_registrations():
    """Store._encode registers under Domain.journal(): an encode that fails part way (a
    65th token, an element past capacity, a non-orddict) leaves no slots behind, and the
    term order afterwards is the order of the surviving slots."""
    from lasp_amd.codec import CapacityError
    dom = Domain(element_capacity=4)
    dom.encode_orset([[(1, [(b"t1", False)]), (3, [(b"t3", False)])]], 4)
    before = (list(dom.elements.terms), [list(t.terms) for t in dom.tokens], list(dom.tok_log))
    order0 = list(dom.elements.order())
    with pytest.raises(CapacityError):
        with dom.journal():
            dom.encode_orset([[(0, [(b"a", False)]), (2, [(b"b", False)]),
                               (5, [(b"c", False)]), (7, [(b"d", False)])]], 4)
    assert (list(dom.elements.terms), [list(t.terms) for t in dom.tokens],
            list(dom.tok_log)) == before
    assert list(dom.elements.order()) == order0
    assert dom.element_slot(5, create=False) == -1
    with pytest.raises(CapacityError):
        with dom.journal():
            for k in range(65):
                dom.token_slot(0, bytes([k]))
    assert list(dom.tokens[0].terms) == [b"t1"]
    with dom.journal():                      # a block that succeeds keeps its slots
        dom.element_slot(2)
    assert dom.size == 3 and len(dom.tokens) == 3
    assert [dom.elements.terms[int(s)] for s in dom.elements.order()] == [1, 2, 3]


def _small_atom_utf8(name: str) -> bytes:
    b = name.encode()
    return bytes([119, len(b)]) + b


def test_dict_refuses_equal_terms_under_other_images(lib):
    """`==` classes: the dictionary keys slots by image bytes, so a term
    `==` to a registered one under another image — 1 and 1.0, {a, 1} and {a, 1.0}, [1] and
    [1.0], an atom in another encoding, 2^64 and 1.8446744073709552e19, -0.0 and 0 — would
    take a second slot where orddict:merge / ordsets:union (lasp_orset.erl:128-134,
    lasp_gset.erl:99-101) see one key.  Its payload gets
    LASPJ_DEC_EQUAL_TERMS and registers nothing; terms that only look alike (2^64 + 1 and
    that float, 0.5 and 1) register normally."""
    from lasp_amd.hostdict import NativeDict
    tok = b"t" * 20
    od = lambda e, t=tok: etf.term_to_binary([(e, [(t, False)])])     # noqa: E731
    pairs = [(1, 1.0), (-3, -3.0), ((Atom("a"), 1), (Atom("a"), 1.0)), ([1, 2], [1.0, 2]),
             (2 ** 64, 1.8446744073709552e19), (0, -0.0), (2 ** 70, float(2 ** 70)),
             (((1,), [2]), ((1.0,), [2.0]))]
    for x, y in pairs:
        d = NativeDict()
        assert list(d.add(_lib.KIND_ORSET, [od(x)])) == [_lib.DEC_OK], x
        n0 = d.info()
        assert list(d.add(_lib.KIND_ORSET, [od(y)])) == [_lib.DEC_EQUAL_TERMS], (x, y)
        assert d.info() == n0
        # the registered image itself is still welcome
        assert list(d.add(_lib.KIND_ORSET, [od(x)])) == [_lib.DEC_OK]
        g = NativeDict()
        assert list(g.add(_lib.KIND_GSET, [etf.term_to_binary([x])])) == [_lib.DEC_OK]
        assert list(g.add(_lib.KIND_GSET, [etf.term_to_binary([y])])) == [_lib.DEC_EQUAL_TERMS]
    # within one payload (not an orddict: 1 < 1.0 is false) and across tokens of an element
    d = NativeDict()
    assert list(d.add(_lib.KIND_ORSET, [etf.term_to_binary([(1, [(tok, False)]),
                                                            (1.0, [(tok, False)])])])) == \
        [_lib.DEC_EQUAL_TERMS]
    assert d.info()[0] == 0
    assert list(d.add(_lib.KIND_ORSET, [etf.term_to_binary([(5, [(7, False)])])])) == [0]
    assert list(d.add(_lib.KIND_ORSET, [etf.term_to_binary([(5, [(7.0, True)])])])) == \
        [_lib.DEC_EQUAL_TERMS]
    # an atom in SMALL_ATOM_UTF8_EXT (an OTP 26 node's image) against ATOM_EXT
    d = NativeDict()
    plain = etf.term_to_binary([(Atom("zed"), [(tok, False)])])
    assert list(d.add(_lib.KIND_ORSET, [plain])) == [0]
    other = plain.replace(bytes([100, 0, 3]) + b"zed", _small_atom_utf8("zed"))
    assert other != plain
    assert list(d.add(_lib.KIND_ORSET, [other])) == [_lib.DEC_EQUAL_TERMS]
    # look-alikes that are not `==` register as separate terms
    for x, y in [(2 ** 64 + 1, 1.8446744073709552e19), (0.5, 1), (1, (1,)), ([1], [[1]]),
                 (b"a", [97]), ([], b"")]:
        d = NativeDict()
        assert list(d.add(_lib.KIND_ORSET, [od(x), od(y)])) == [0, 0], (x, y)
        assert d.info()[0] == 2


@settings(max_examples=300 * SOAK, deadline=None, suppress_health_check=[HealthCheck.too_slow])
@given(TERM, TERM)
def test_dict_equal_terms_iff_compare_equal(lib, a, b):
    """The `==` class check agrees with the comparator: b registers after a exactly when
    the two are not `==` or have the same image."""
    from lasp_amd.hostdict import NativeDict
    d = NativeDict()
    ia, ib = etf.encode(a), etf.encode(b)
    pa = bytes([131, 108, 0, 0, 0, 1]) + ia + bytes([106])
    pb = bytes([131, 108, 0, 0, 0, 1]) + ib + bytes([106])
    assert list(d.add(_lib.KIND_GSET, [pa])) == [0]
    st_ = d.add(_lib.KIND_GSET, [pb])[0]
    same_class = compare(lib, a, b) == 0 and ia != ib
    assert st_ == (_lib.DEC_EQUAL_TERMS if same_class else _lib.DEC_OK), (a, b)


def test_domain_refuses_equal_terms():
    """The Python Domain (the device store's dictionaries) refuses a second term of one
    `==` class too, instead of letting the first-seen term stand for both: the store then
    raises Unsupported."""
    from lasp_amd.codec import CapacityError, EqualTerms
    dom = Domain()
    dom.element_slot(1)
    assert dom.element_slot(1) == 0
    with pytest.raises(EqualTerms):
        dom.element_slot(1.0)
    assert issubclass(EqualTerms, CapacityError)
    es = dom.element_slot((Atom("a"), 2))
    with pytest.raises(EqualTerms):
        dom.element_slot((Atom("a"), 2.0))
    dom.token_slot(es, 3)
    with pytest.raises(EqualTerms):
        dom.token_slot(es, 3.0)
    # true / Atom("true") are one atom: no refusal
    t = dom.element_slot(True)
    assert dom.element_slot(Atom("true")) == t
    with pytest.raises(EqualTerms):
        dom.encode_orset([[(1.0, [(b"x" * 20, False)])]], 16)
