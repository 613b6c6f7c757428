"""The lasp_gset NIF entry points and the device-resident variables (include/laspj.h
"NIF entry points", "resident variables"; lasp_amd/csrc/laspj_nif.hip), against the oracle.

G-Set: merge/2 = ordsets:union (lasp_gset.erl:99-101), value/1 = ordsets:to_list
(:74-76), equal/2 = == (:103-105), is_(strict_)inflation (lasp_lattice.erl:137-140,
212-215) — term_to_binary images in, the oracle's image / boolean out, or FALLBACK for a
list that is not an ordset.

Variables: `#dv.value` (include/lasp.hrl:60-63) kept on the device; bind/3
(lasp_core.erl:291-312) ships only the incoming value and answers the status (no-op when
`Value0 =:= Value`, else merge + write), read / value / threshold_met
(lasp_lattice.erl:62-75) answer from the resident cells, write/4 (:839-844) replaces the
value or holds an unrepresentable one as its image; a dictionary reset writes resident
variables out to their images and they come back on their next call.
"""

import functools
import random

import pytest

from oracle import etf as oetf
from oracle import gset as ogset
from oracle import lattice as olat
from oracle import orset as oorset
from oracle import otp
from oracle.terms import Atom, compare, exact_eq

OK, FALLBACK = 0, 1
_key = functools.cmp_to_key(compare)

pytestmark = pytest.mark.gpu


def _tb(t) -> bytes:
    return oetf.term_to_binary(t)


def _ctx():
    from lasp_amd import engine
    return engine.Context(0)


def _tokens(rng, n, size=20):
    return [bytes(rng.getrandbits(8) for _ in range(size)) for _ in range(n)]


def _gpool(rng, n=60):
    pool = list(range(0, 200, 3)) + [Atom(f"g{k}") for k in range(10)] + \
        [bytes([k]) * 3 for k in range(10)] + [(k, Atom("x")) for k in range(5)] + \
        list(range(300, 340))
    return pool


def _gset(rng, pool, p=0.4):
    return otp.lists_usort([x for x in pool if rng.random() < p])


# ------------------------------------------------------------------ lasp_gset

def test_gset_nif_answers_match_oracle():
    ctx = _ctx()
    try:
        rng = random.Random(3)
        pool = _gpool(rng)
        for k in range(30):
            a, b = _gset(rng, pool), _gset(rng, pool)
            m = ogset.merge(a, b)
            assert ctx.nif_merge(_tb(a), _tb(b), kind="gset") == (OK, _tb(m)), k
            assert ctx.nif_value(_tb(a), kind="gset") == (OK, _tb(ogset.value(a)))
            same = a if k % 3 == 0 else b
            assert ctx.nif_equal(_tb(a), _tb(same), kind="gset") == (OK, ogset.equal(a, same))
            cur = m if k % 2 else b
            assert ctx.nif_inflation(_tb(a), _tb(cur), kind="gset") == \
                (OK, olat.is_inflation("lasp_gset", a, cur))
            cur = a if k % 4 == 0 else cur
            assert ctx.nif_inflation(_tb(a), _tb(cur), strict=True, kind="gset") == \
                (OK, olat.is_strict_inflation("lasp_gset", a, cur))
        # empty sets, all-byte integers (STRING_EXT images) and merges of many pairs
        assert ctx.nif_merge(_tb([]), _tb([]), kind="gset") == (OK, _tb([]))
        assert ctx.nif_merge(_tb([1, 2, 250]), _tb([3]), kind="gset") == (OK, _tb([1, 2, 3, 250]))
        assert ctx.nif_inflation(_tb([]), _tb([5]), strict=True, kind="gset") == (OK, True)
        pairs = [(_gset(rng, pool), _gset(rng, pool)) for _ in range(24)]
        got = ctx.nif_merge_many([(_tb(a), _tb(b)) for a, b in pairs], kind="gset")
        assert got == [(OK, _tb(ogset.merge(a, b))) for a, b in pairs]
        # long sets (the split writer: chunks of 256 term-order slots over the chip), and
        # value/1 of a 10k-element OR-Set image (its answer is a G-Set image)
        big_a, big_b = list(range(0, 20000, 2)), list(range(0, 30000, 3)) + [Atom("z")]
        assert ctx.nif_merge(_tb(big_a), _tb(big_b), kind="gset") == \
            (OK, _tb(ogset.merge(big_a, big_b)))
        longs = [(big_a, big_b), (big_b[:3000], big_a[::7]), ([], big_a), (big_b, [])]
        assert ctx.nif_merge_many([(_tb(x), _tb(y)) for x, y in longs], kind="gset") == \
            [(OK, _tb(ogset.merge(x, y))) for x, y in longs]
        o = [(e, [(b"A" + e.to_bytes(19, "big"), e % 7 == 0)]) for e in range(10000)]
        assert ctx.nif_value(_tb(o)) == (OK, _tb(oorset.value(o)))
        # (the value pass clears its decoded cells behind it: the next calls decode into
        # them without a memset)
        o2 = [(e, [(b"A" + e.to_bytes(19, "big"), e % 5 == 0)]) for e in range(0, 10000, 3)]
        assert ctx.nif_value(_tb(o2)) == (OK, _tb(oorset.value(o2)))
        assert ctx.nif_merge(_tb(o2), _tb(o)) == (OK, _tb(oorset.merge(o2, o)))
        assert ctx.nif_value(_tb(o)) == (OK, _tb(oorset.value(o)))
        # a resident variable's value/1 twice: its cells stay
        v = ctx.var("orset")
        v.write(_tb(o))
        assert v.value() == (OK, _tb(oorset.value(o)))
        assert v.value() == (OK, _tb(oorset.value(o)))
        assert v.read() == (OK, _tb(o))
    finally:
        ctx.close()


def test_gset_nif_fallbacks():
    """Lists that are not ordsets in term order (the reference's ordsets:union runs as
    written on them: SURVEY.md Appendix A / B2), improper lists, non-lists and `==`
    classes answer FALLBACK; value/1 is the identity on any term."""
    ctx = _ctx()
    try:
        good = [1, 5, Atom("a")]
        bad = {
            "unsorted": [5, 1],
            "repeated": [1, 1],
            "not a list": Atom("a"),
            "int and float": [1, 1.0],
        }
        assert ctx.nif_merge(_tb(good), _tb(good), kind="gset") == (OK, _tb(good))
        for name, v in bad.items():
            assert ctx.nif_merge(_tb(good), _tb(v), kind="gset") == (FALLBACK, None), name
            assert ctx.nif_equal(_tb(v), _tb(good), kind="gset") == (FALLBACK, None), name
            assert ctx.nif_inflation(_tb(good), _tb(v), kind="gset") == (FALLBACK, None), name
            assert ctx.nif_value(_tb(v), kind="gset") == (OK, _tb(v))
        # 1.0 after 1 holds a slot: FALLBACK (ordsets:union([1], [1.0]) keeps 1)
        v, ans = ctx.nif_merge(_tb([1]), _tb([1.0]), kind="gset")
        assert (v, ans) == (FALLBACK, None) or ans == _tb(ogset.merge([1], [1.0]))
        improper = _tb(good)[:-1] + bytes([97, 3])
        assert ctx.nif_merge(_tb(good), improper, kind="gset") == (FALLBACK, None)
    finally:
        ctx.close()


# ------------------------------------------------------------------ resident variables

def _orset(rng, elems, pool, p=0.6, pflag=0.3):
    s = []
    for e in elems:
        if rng.random() < p:
            ts = pool[e]
            k = rng.randint(1, len(ts))
            toks = sorted(rng.sample(ts, k), key=_key)
            s.append((e, [(t, rng.random() < pflag) for t in toks]))
    return s


def _universe(rng, n):
    elems = sorted(list(range(n // 2)) + [Atom(f"e{k}") for k in range(n // 4)] +
                   [f"b{k}".encode() for k in range(n - n // 2 - n // 4)], key=_key)
    return elems, {e: _tokens(rng, 5) for e in elems}


def _bind_oracle(type_, value0, value):
    """lasp_core:bind/3 (lasp_core.erl:291-312) on canonical values: (status, Value0')."""
    mod = oorset if type_ == "lasp_orset" else ogset
    if exact_eq(value0, value):
        return 0, value0
    merged = mod.merge(value0, value)
    assert olat.is_inflation(type_, value0, merged)      # canonical merges always inflate
    return 1, merged


def test_var_bind_sequence_matches_oracle():
    """bind/3 on a resident OR-Set variable, 80 times: repeated values (the no-op), new
    tokens on known elements (a remote update), new elements, removals seen elsewhere,
    []; after each: the status, read/0 (the value's image), value/1 and threshold_met
    with earlier values as thresholds (strict and not) agree with the oracle."""
    ctx = _ctx()
    try:
        rng = random.Random(21)
        elems, pool = _universe(rng, 60)
        var = ctx.var("orset")
        cur = []
        assert var.read() == (OK, _tb([]))
        assert var.bind(_tb([])) == (OK, 0)                 # [] =:= []: no-op
        history = [[]]
        for k in range(80):
            if k % 9 == 4:
                val = cur                                   # Value0 =:= Value
            elif k % 11 == 7:
                e = rng.choice(elems)
                pool[e].append(bytes(rng.getrandbits(8) for _ in range(20)))
                val = _orset(rng, elems, pool, p=0.3)
            else:
                val = _orset(rng, elems, pool)
            want_st, cur_next = _bind_oracle("lasp_orset", cur, val)
            assert var.bind(_tb(val)) == (OK, want_st), k
            cur = cur_next
            assert var.read() == (OK, _tb(cur)), k
            if k % 5 == 0:
                assert var.value() == (OK, _tb(oorset.value(cur)))
                th = rng.choice(history)
                assert var.threshold(_tb(th)) == (OK, olat.threshold_met("lasp_orset", cur, th))
                assert var.threshold(_tb(th), strict=True) == \
                    (OK, olat.threshold_met("lasp_orset", cur, ("strict", th)))
                history.append(cur)
        assert var.resident
        # a threshold the variable has not reached (an element it never saw)
        th = [(Atom("zz_new"), [(b"\x01" * 20, False)])]
        assert var.threshold(_tb(th)) == (OK, False)
        var.close()
    finally:
        ctx.close()


def test_var_gset_bind_read_threshold():
    ctx = _ctx()
    try:
        rng = random.Random(5)
        pool = _gpool(rng)
        var = ctx.var("gset")
        cur = []
        for k in range(40):
            val = cur if k % 7 == 3 else _gset(rng, pool, p=0.2)
            want_st, cur = _bind_oracle("lasp_gset", cur, val)
            assert var.bind(_tb(val)) == (OK, want_st), k
            assert var.read() == (OK, _tb(cur))
            assert var.value() == (OK, _tb(cur))
            th = _gset(rng, pool, p=0.05)
            assert var.threshold(_tb(th)) == (OK, olat.threshold_met("lasp_gset", cur, th))
            assert var.threshold(_tb(cur), strict=True) == (OK, False)
        var.close()
    finally:
        ctx.close()


def test_var_bind_many_and_fallbacks():
    """Eight variables bound in one device pass (laspj_var_etf_bind_many); an operand the
    columnar form does not take answers FALLBACK and leaves its variable as it was; a
    `==`-equal element under another image (1.0 after 1) likewise; a variable named twice
    or owned by another context is an argument error."""
    from lasp_amd import _lib
    ctx = _ctx()
    try:
        rng = random.Random(8)
        elems, pool = _universe(rng, 40)
        vs = [ctx.var("orset") for _ in range(8)]
        cur = [[] for _ in vs]
        for rnd in range(6):
            vals = [_orset(rng, elems, pool) for _ in vs]
            if rnd == 3:
                vals[2] = cur[2]
                vals[5] = [(2, [(b"x" * 20, False)]), (1, [(b"y" * 20, False)])]   # keys descend
            got = ctx.var_bind_many(list(zip(vs, [_tb(v) for v in vals])))
            for i, v in enumerate(vs):
                if rnd == 3 and i == 5:
                    assert got[i][0] == FALLBACK
                    continue
                st, cur[i] = _bind_oracle("lasp_orset", cur[i], vals[i])
                assert got[i] == (OK, st), (rnd, i)
            for i, v in enumerate(vs):
                assert v.read() == (OK, _tb(cur[i])), (rnd, i)
        w = ctx.var("orset")
        assert w.bind(_tb([(1, [(b"t" * 20, False)])])) == (OK, 1)
        assert w.bind(_tb([(1.0, [(b"u" * 20, False)])]))[0] == FALLBACK
        assert w.read() == (OK, _tb([(1, [(b"t" * 20, False)])]))
        with pytest.raises(_lib.LaspjError):
            ctx.var_bind_many([(vs[0], _tb([])), (vs[0], _tb([]))])
        other = _ctx()
        try:
            ov = other.var("orset")
            with pytest.raises(_lib.LaspjError):
                ctx.var_bind_many([(vs[0], _tb([])), (ov, _tb([]))])
            ov.close()
        finally:
            other.close()
    finally:
        ctx.close()


def test_var_write_unrepresentable_is_held_as_its_image():
    """write/4 of a value the columnar form cannot hold (an element with 65 tokens whose
    images are not all of one length: past 64 the namespace's wide cells need fixed-width
    token templates) keeps it as its image: read answers it, bind / threshold / value
    answer FALLBACK (the NIF runs the reference's clause over the read term), and a
    representable write brings the variable back to the device."""
    ctx = _ctx()
    try:
        rng = random.Random(9)
        toks = sorted(_tokens(rng, 70))
        mixed = sorted(toks[:64] + [toks[64] + b"xy"], key=_key)
        big = [(1, [(t, bool(k % 3 == 0)) for k, t in enumerate(mixed)])]
        var = ctx.var("orset")
        assert var.write(_tb(big)) == FALLBACK
        assert not var.resident
        assert var.read() == (OK, _tb(big))
        assert var.bind(_tb([(2, [(toks[66], False)])])) == (FALLBACK, 0)
        assert var.threshold(_tb([]))[0] == FALLBACK
        assert var.value() == (FALLBACK, None)
        small = [(1, [(toks[0], True)]), (2, [(toks[66], False)])]
        assert var.write(_tb(small)) == OK
        assert var.resident
        assert var.read() == (OK, _tb(small))
        assert var.bind(_tb([(3, [(toks[67], False)])])) == (OK, 1)
        assert var.read() == (OK, _tb(oorset.merge(small, [(3, [(toks[67], False)])])))
        var.close()
    finally:
        ctx.close()


def test_var_survives_a_dictionary_reset():
    """The image calls' dictionary resets (an element whose 64 token slots earlier calls used
    up) without touching the variables, whose namespaces are their own.  Replicas writing
    values whose tokens on one element add up past 64 widen their namespace instead; every
    variable keeps binding exactly as the oracle does."""
    ctx = _ctx()
    try:
        rng = random.Random(10)
        elems, pool = _universe(rng, 30)
        vs = [ctx.var("orset") for _ in range(3)]
        cur = []
        for v in vs:
            val = _orset(rng, elems, pool)
            assert v.bind(_tb(val))[0] == OK
            cur.append(val)
        s0 = ctx.nif_stats()
        for k in range(4):                      # 4 x 40 distinct tokens on element 1
            toks = sorted(_tokens(rng, 40))
            a = [(1, [(t, False) for t in toks[:20]])]
            b = [(1, [(t, bool(i % 2)) for i, t in enumerate(toks[20:])])]
            assert ctx.nif_merge(_tb(a), _tb(b)) == (OK, _tb(oorset.merge(a, b)))
        s1 = ctx.nif_stats()
        assert s1["dict_resets"] > s0["dict_resets"]
        assert s1["vars_spilled"] == s0["vars_spilled"]
        for i, v in enumerate(vs):
            assert v.resident
            assert v.read() == (OK, _tb(cur[i])), i
        # replicas in one namespace: 40 + 40 tokens on element 1 do not fit 64 slots; the
        # namespace goes wide (k pairs per cell) and nothing is written out
        r0 = vs[0]
        r1 = r0.replica()
        toks = sorted(_tokens(rng, 80))
        w1 = [(1, [(t, False) for t in toks[:40]])]
        w2 = [(1, [(t, True) for t in toks[40:]])]
        assert r1.write(_tb(w1)) == OK
        assert r0.write(_tb(w2)) == OK
        s2 = ctx.nif_stats()
        assert s2["vars_spilled"] == s1["vars_spilled"]
        assert s2["dict_resets"] == s1["dict_resets"]
        assert r1.read() == (OK, _tb(w1))
        assert r1.bind(_tb(w2)) == (OK, 1)
        assert r1.read() == (OK, _tb(oorset.merge(w1, w2)))
        cur[0] = w2
        for i, v in enumerate(vs):
            assert v.read() == (OK, _tb(cur[i])), i
            val = _orset(rng, elems, pool)
            st, cur[i] = _bind_oracle("lasp_orset", cur[i], val)
            assert v.bind(_tb(val)) == (OK, st)
            assert v.read() == (OK, _tb(cur[i]))
    finally:
        ctx.close()


def test_var_config1_bind():
    """BASELINE configs[0]'s shape: a resident replica A (10k elements, 1-3 tokens each)
    binds replica B (its 10 % removals seen elsewhere); the value read back is the
    oracle's merge, and binding B again is a write that changes nothing (B is not
    Value0)."""
    ctx = _ctx()
    try:
        rng = random.Random(77)
        ta = lambda e: b"A" + e.to_bytes(4, "big") + bytes(15)   # noqa: E731
        tb = lambda e: b"B" + e.to_bytes(4, "big") + bytes(15)   # noqa: E731
        A = [(e, [(ta(e), False)]) for e in range(10_000)]
        rm = set(rng.sample(range(10_000), 1000))
        B = [(e, [(tb(e), e in rm)]) for e in range(10_000)]
        var = ctx.var("orset")
        assert var.bind(_tb(A)) == (OK, 1)
        assert var.bind(_tb(B)) == (OK, 1)
        want = oorset.merge(A, B)
        assert var.read() == (OK, _tb(want))
        assert var.bind(_tb(B)) == (OK, 1)
        assert var.read() == (OK, _tb(want))
        assert var.bind(_tb(want)) == (OK, 0)
        var.close()
    finally:
        ctx.close()


def test_nif_and_var_fuzz_mutated_images():
    """Mutated term_to_binary images (truncated, a bit flipped, junk appended, a tag byte
    replaced) into merge / equal / value and into a resident variable's bind: each call
    answers FALLBACK, raises an error status, or answers OK with the oracle's answer on the
    terms the images decode to; a variable's value stays the oracle's after every bind that
    answered (a failed decode leaves it untouched)."""
    from lasp_amd import _lib
    ctx = _ctx()
    try:
        rng = random.Random(57)
        elems, pool = _universe(rng, 40)
        A = _orset(rng, elems, pool)
        B = _orset(rng, elems, pool)

        def mutate(img):
            b = bytearray(img)
            k = rng.randrange(4)
            if k == 0 and len(b) > 2:
                return bytes(b[:rng.randrange(1, len(b))])
            if k == 1:
                i = rng.randrange(len(b))
                b[i] ^= 1 << rng.randrange(8)
                return bytes(b)
            if k == 2:
                return bytes(b) + bytes(rng.getrandbits(8) for _ in range(rng.randint(1, 6)))
            i = rng.randrange(1, len(b))
            b[i] = rng.choice([97, 98, 100, 104, 106, 107, 108, 109, 110, 115, 118, 119])
            return bytes(b)

        def decoded(img):
            try:
                return True, oetf.binary_to_term(img)
            except Exception:
                return False, None

        var = ctx.var("orset")
        assert var.bind(_tb(A)) == (OK, 1)
        cur = A
        answered = 0
        for n in range(1500):
            ma = mutate(_tb(B))
            op = n % 4
            try:
                if op == 0:
                    verd, img = ctx.nif_merge(_tb(A), ma)
                elif op == 1:
                    verd, res = ctx.nif_equal(_tb(A), ma)
                elif op == 2:
                    verd, img = ctx.nif_value(ma)
                else:
                    verd, st = var.bind(ma)
            except _lib.LaspjError:
                continue
            assert verd in (OK, FALLBACK)
            if verd != OK:
                continue
            ok, tb_ = decoded(ma)
            assert ok, (op, ma)
            if op == 0:
                assert exact_eq(oetf.binary_to_term(img), oorset.merge(A, tb_))
            elif op == 1:
                assert res == oorset.equal(A, tb_)
            elif op == 2:
                assert exact_eq(oetf.binary_to_term(img), oorset.value(tb_))
            else:
                want_st, cur2 = _bind_oracle("lasp_orset", cur, tb_)
                assert st == want_st
                cur = cur2
            answered += 1
        assert answered > 0
        verd, img = var.read()
        assert verd == OK and exact_eq(oetf.binary_to_term(img), cur)
    finally:
        ctx.close()
