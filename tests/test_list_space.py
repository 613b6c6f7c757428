"""The host rank tables of list values (lasp_amd/lists.py ListSpace) kept incrementally:
token labels must order token ids exactly as Erlang term order does (equal terms equal
labels), and the device copy must hold what the host holds after every refresh —
checked against a full sort, with ascending runs that use gaps up, random inserts,
`==`-equal terms in different slots and bulk growth.  CPU only: a recording stand-in
replaces the device buffers."""
import random

import numpy as np
import pytest

from lasp_amd import lists as L
from lasp_amd.codec import Domain, EqualTerms, _Dict
from lasp_amd.terms import term_cmp, term_key


class _H:
    value = 1


class _Buf:
    def __init__(self, n):
        self.nbytes = n
        self.h = _H()
        self.mem = np.zeros((n,), dtype=np.uint8)

    def upload(self, arr, offset=0):
        b = np.ascontiguousarray(arr).view(np.uint8).reshape(-1)
        self.mem[offset:offset + len(b)] = b


class _Ctx:
    def buffer(self, n):
        return _Buf(n)


def _check(sp, d):
    o = sp.order()
    K = max(1, d.size)
    kr = sp._kbuf.mem[:4 * K].view(np.uint32)
    eo = sorted(range(d.size), key=lambda i: term_key(d.elements.terms[i]))
    assert [int(x) for x in np.argsort(kr[:d.size], kind="stable")] == eo
    gr = sp._gbuf.mem.view(np.uint32)
    assert o.ntokens == 64 * K and len(gr) >= 64 * K
    toks = [(64 * e + k, t) for e in range(d.size) for k, t in enumerate(d.tokens[e].terms)]
    for _ in range(400 if len(toks) > 1 else 0):
        (g1, t1), (g2, t2) = random.sample(toks, 2)
        c = term_cmp(t1, t2)
        l1, l2 = int(gr[g1]), int(gr[g2])
        assert 0 < l1 < (1 << 31) and 0 < l2 < (1 << 31)
        assert (l1 > l2) - (l1 < l2) == c, (t1, t2, l1, l2)


def test_token_labels_follow_term_order():
    random.seed(7)
    for trial in range(6):
        d = Domain(element_capacity=1 << 16)
        sp = L.ListSpace(_Ctx(), d, tokens=True)
        nxt = 0
        for step in range(60):
            mode = random.random()
            if mode < 0.3:                      # ascending appends (use gaps up)
                for _ in range(random.randint(1, 400)):
                    e = d.element_slot(random.randint(0, 300))
                    if len(d.tokens[e]) < 64:
                        d.token_slot(e, nxt.to_bytes(8, "big"))
                    nxt += 1
            elif mode < 0.6:                    # random binaries and numbers, == pairs
                for _ in range(random.randint(1, 50)):
                    e = d.element_slot(random.randint(0, 300))
                    if len(d.tokens[e]) < 62:
                        v = random.randint(0, 1000)
                        d.token_slot(e, v)
                        # (the second image of a `==` class is refused, not given a slot)
                        with pytest.raises(EqualTerms):
                            d.token_slot(e, float(v))
                        d.token_slot(e, v + 0.5)
                        d.token_slot(e, bytes(random.randrange(256) for _ in range(3)))
            elif mode < 0.63:                   # bulk growth
                for _ in range(5000):
                    e = d.element_slot(random.randint(0, 2000))
                    if len(d.tokens[e]) < 64:
                        d.token_slot(e, random.random())
            _check(sp, d)
        assert sp._relabels >= 1


def test_dict_order_incremental_matches_sort():
    random.seed(3)
    for trial in range(100):
        dd = _Dict(1 << 20)
        for _ in range(150):
            # (a float `==` to a registered int is refused: EqualTerms, no slot)
            try:
                dd.slot(random.choice([random.randint(0, 40), float(random.randint(0, 40)),
                                       (1, random.randint(0, 4)), bytes([random.randint(0, 9)])]))
            except EqualTerms:
                pass
            if random.random() < 0.3:
                dd.order()
            if random.random() < 0.01:
                for _ in range(1100):
                    dd.slot(random.random())
        want = sorted(range(len(dd.terms)), key=lambda i: term_key(dd.terms[i]))
        assert list(dd.order()) == want


def test_wide_domain_list_tables_hold_token_slots_below_64():
    """A Store domain with more than 64 token slots per element (wide OR-Set cells): list
    values name 64 token slots per element (g = 64 e + k), so the rank tables place slots
    0..63 only — bulk and incremental paths — the from_set token-order rows list those,
    and encoding a list value that names a later slot raises CapacityError (the store's
    Unsupported) instead of aliasing another element's token id."""
    from lasp_amd.codec import CapacityError
    random.seed(11)
    for bulk in (False, True):
        d = Domain(element_capacity=1 << 12, token_capacity=64 * 4)
        sp = L.ListSpace(_Ctx(), d, tokens=True)
        nel = 80 if bulk else 2
        for e in range(nel):
            es = d.element_slot(e)
            ks = list(range(100))
            random.shuffle(ks)
            for k in ks:
                d.token_slot(es, (e, k))
        o = sp.order()
        assert o.ntokens == 64 * d.size
        gr = sp._gbuf.mem.view(np.uint32)
        for e in range(nel):
            terms = d.tokens[e].terms[:64]
            labs = [int(gr[64 * e + k]) for k in range(64)]
            assert all(lab > 0 for lab in labs)
            assert sorted(range(64), key=lambda k: labs[k]) == \
                sorted(range(64), key=lambda k: term_key(terms[k]))
        _eb, _n, tb = sp.set_orders(d.size)
        row = tb.mem[64 * 0: 64 * 1]
        want = [k for k in d.tokens[0].order() if k < 64]
        assert [int(x) for x in row[:len(want)]] == want and len(want) == 64
    late = next(t for k, t in enumerate(d.tokens[0].terms) if k >= 64)
    with pytest.raises(CapacityError):
        L.encode(d, [(0, [(late, False)])], False)
    with pytest.raises(CapacityError):
        d.encode_orset([[(0, [(late, False)])]], d.size)
    assert d.orset_words([[(0, [(late, False)])]]) == 2
    early = d.tokens[0].terms[3]
    s = sorted([(early, False), (late, True)], key=lambda x: term_key(x[0]))
    cells = d.encode_orset_wide([[(0, s)]], d.size, 2)
    assert d.decode_orset_wide(cells[0]) == [(0, s)]
