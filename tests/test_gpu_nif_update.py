"""lasp_core:update/4 on resident variables (laspj_var_etf_update) and per-variable token
namespaces (include/laspj.h "resident variables"; lasp_amd/csrc/laspj_nif.hip), against the
oracle.

update/4 (lasp_core.erl:283-287) is Type:update(Op, Actor, Value0) then bind/3 of the result:
OR-Set ops {add, E} (a token minted by unique/1, lasp_orset.erl:261-262), {add_by_token, T,
E}, {add_all, Es}, {remove, E}, {remove_all, Es}, {update, Ops} (:99-117, 222-259) and G-Set
{add, E}, {add_all, Es} (lasp_gset.erl:84-88) run on the device cells; a failed precondition
answers {error, {precondition, {not_present, E}}} and voids the whole call.  Minted tokens
come back from the call, so the oracle replays the same update with them.

Namespaces: each variable's dictionary holds its own value's terms, so a hundred variables
holding element 1 with their own tokens never exhaust its 64 slots (include/lasp.hrl:60-63);
replicas created in one namespace know each other's tokens, so a bind of a replica's state
after an update decodes in one device pass.
"""

import functools
import random

import pytest

from oracle import etf as oetf
from oracle import gset as ogset
from oracle import lattice as olat
from oracle import orset as oorset
from oracle.terms import Atom, compare, exact_eq

OK, FALLBACK = 0, 1
UPD_OK, NOT_PRESENT = 0, 1
A = Atom
_key = functools.cmp_to_key(compare)

pytestmark = pytest.mark.gpu
SOAK = int(__import__("os").environ.get("LASPJ_SOAK", "1"))   # x rounds for a soak run


def _tb(t) -> bytes:
    return oetf.term_to_binary(t)


def _ctx():
    from lasp_amd import engine
    return engine.Context(0)


def _oracle_update(mod, op, state, minted):
    """Type:update/3 on the oracle with the tokens the device minted, in op order."""
    it = iter(minted)
    if mod is ogset:
        return ogset.update(op, A("a"), state)
    return oorset.update(op, A("a"), state, tokens=lambda _actor: next(it))


def _elements(rng):
    return list(range(12)) + [A(f"e{k}") for k in range(6)] + [f"s{k}".encode() for k in range(4)] + \
        [(k, A("t")) for k in range(3)]


def _rand_op(rng, elems, toks, depth=0):
    k = rng.randrange(9 if depth == 0 else 7)
    e = rng.choice(elems)
    if k in (0, 1):
        return (A("add"), e)
    if k == 2:
        return (A("add_by_token"), rng.choice(toks), e)
    if k == 3:
        return (A("add_all"), [rng.choice(elems) for _ in range(rng.randint(0, 4))])
    if k in (4, 5):
        return (A("remove"), e)
    if k == 6:
        return (A("remove_all"), [rng.choice(elems) for _ in range(rng.randint(0, 3))])
    return (A("update"), [_rand_op(rng, elems, toks, depth + 1) for _ in range(rng.randint(0, 4))])


def test_var_update_random_ops_match_oracle():
    """300 random update/4 calls on a resident OR-Set variable (every op form, nested
    {update, Ops}, removes of absent elements, re-adds by a known token): the result, the
    failing element and the value read back agree with lasp_orset:update/3 replayed on the
    oracle with the minted tokens; value/1 and threshold_met agree along the way."""
    ctx = _ctx()
    try:
        rng = random.Random(61)
        elems = _elements(rng)
        toks = [bytes(rng.getrandbits(8) for _ in range(20)) for _ in range(6)] + [A("tk"), 7]
        var = ctx.var("orset")
        cur = []
        history = [[]]
        counts = {UPD_OK: 0, NOT_PRESENT: 0}
        for k in range(300):
            op = _rand_op(rng, elems, toks)
            verd, res, err, minted = var.update(_tb(op))
            assert verd == OK, (k, op)
            assert all(len(t) == 20 for t in minted)
            want = _oracle_update(oorset, op, cur, minted)
            if want[0] == "ok":
                assert res == UPD_OK, (k, op)
                cur = want[1]
            else:
                assert res == NOT_PRESENT, (k, op)
                assert exact_eq(oetf.binary_to_term(bytes([131]) + err), want[1][1][1]), (k, op)
            counts[res] += 1
            if k % 7 == 0 or res == NOT_PRESENT:
                assert var.read() == (OK, _tb(cur)), (k, op)
            if k % 25 == 0:
                assert var.value() == (OK, _tb(oorset.value(cur)))
                th = rng.choice(history)
                assert var.threshold(_tb(th)) == (OK, olat.threshold_met("lasp_orset", cur, th))
                history.append(cur)
        assert counts[UPD_OK] > 100 and counts[NOT_PRESENT] >= 5
        assert var.read() == (OK, _tb(cur))
        # a bind after updates: the merge of a state with the variable's own tokens
        other = oorset.merge(cur, [(A("zz"), [(b"\x07" * 20, False)])])
        assert var.bind(_tb(other)) == (OK, 1)
        assert var.read() == (OK, _tb(other))
    finally:
        ctx.close()


def test_var_update_preconditions_void_the_call():
    """remove_elems / apply_ops stop at the first absent element and the reference returns
    the error, not a state (lasp_orset.erl:232-259): nothing of the call lands, including
    adds before the failing remove; an element added earlier in the same call is present."""
    ctx = _ctx()
    try:
        var = ctx.var("orset")
        t1, t2 = b"\x01" * 20, b"\x02" * 20
        assert var.update(_tb((A("add_by_token"), t1, 1)))[:2] == (OK, UPD_OK)
        before = [(1, [(t1, False)])]
        for op, bad in (((A("remove"), 2), 2),
                        ((A("remove_all"), [1, 2, 3]), 2),
                        ((A("update"), [(A("add_by_token"), t2, 5), (A("remove"), 9)]), 9),
                        ((A("update"), [(A("add"), 4), (A("remove_all"), [1, 4, 6])]), 6)):
            verd, res, err, _m = var.update(_tb(op))
            assert (verd, res) == (OK, NOT_PRESENT), op
            assert oetf.binary_to_term(bytes([131]) + err) == bad
            assert var.read() == (OK, _tb(before)), op
        # add then remove of a new element in one call: present by the add
        verd, res, _e, _m = var.update(_tb((A("update"), [(A("add_by_token"), t2, 5),
                                                          (A("remove"), 5)])))
        assert (verd, res) == (OK, UPD_OK)
        want = oorset.merge(before, [(5, [(t2, True)])])
        assert var.read() == (OK, _tb(want))
        # a re-add by a known token clears its removed flag (orddict:store(Token, false, ..))
        assert var.update(_tb((A("add_by_token"), t2, 5)))[:2] == (OK, UPD_OK)
        assert var.read() == (OK, _tb(oorset.merge(before, [(5, [(t2, False)])])))
    finally:
        ctx.close()


def test_var_update_gset_and_fallbacks():
    """G-Set add / add_all (ordsets:add_element / union with from_list) against the oracle;
    ops no clause takes (an unknown atom, a G-Set remove, a non-list add_all, an improper
    list), a term `==` to a held one under another image (1.0 after 1), and — once an
    element's 65th token has made the namespace wide — a token image of another length
    answer FALLBACK and leave the value as it was."""
    ctx = _ctx()
    try:
        rng = random.Random(5)
        g = ctx.var("gset")
        cur = []
        for k in range(60):
            if k % 3 == 0:
                op = (A("add_all"), [rng.randrange(300) for _ in range(rng.randint(0, 6))] +
                      ([A(f"a{k}")] if k % 2 else []))
            else:
                op = (A("add"), rng.choice([rng.randrange(300), A(f"g{k % 5}"), (k % 4, b"x")]))
            verd, res, err, minted = g.update(_tb(op))
            assert (verd, res, minted) == (OK, UPD_OK, []), op
            cur = ogset.update(op, A("a"), cur)[1]
            assert g.read() == (OK, _tb(cur)), (k, op)
        assert g.update(_tb((A("add"), 1)))[:2] == (OK, UPD_OK)
        cur = ogset.update((A("add"), 1), A("a"), cur)[1]
        for op in ((A("remove"), 1), (A("add_all"), A("x")), (A("nope"), 1), (A("add"), 1.0)):
            assert g.update(_tb(op))[0] == FALLBACK, op
            assert g.read() == (OK, _tb(cur))
        v = ctx.var("orset")
        assert v.update(_tb((A("add_by_token"), b"t" * 20, 1)))[:2] == (OK, UPD_OK)
        state = v.read()[1]
        improper = _tb((A("add_all"), [1, 2]))[:-1] + bytes([97, 3])
        for img in (_tb((A("add"), 1.0)), _tb((A("bogus"), 1)), _tb((A("add_by_token"), 1)),
                    _tb((A("update"), [(A("add"), 2), (A("frob"), 3)])), improper,
                    _tb((A("remove"), 1.0))):
            assert v.update(img)[0] == FALLBACK, img
            assert v.read() == (OK, state)
        # 63 more tokens on element 1 fit; the 65th widens the namespace and fits too
        for k in range(64):
            assert v.update(_tb((A("add"), 1)))[:2] == (OK, UPD_OK), k
        verd, img = v.read()
        assert verd == OK and len(oetf.binary_to_term(img)[0][1]) == 65
        # a wide namespace's tokens are of one image length
        assert v.update(_tb((A("add_by_token"), b"t" * 21, 1)))[0] == FALLBACK
        assert v.read() == (OK, img)
    finally:
        ctx.close()


def test_namespaces_hundred_variables_share_an_element():
    """A vnode's 100 variables each add element 1 three times (300 distinct tokens for one
    element across the context): no dictionary reset, no FALLBACK, and each value is its
    own oracle state; binds of states carrying other variables' tokens stay in their own
    namespaces."""
    ctx = _ctx()
    try:
        s0 = ctx.nif_stats()
        vs = [ctx.var("orset") for _ in range(100)]
        cur = [[] for _ in vs]
        for rnd in range(3):
            for i, v in enumerate(vs):
                verd, res, _e, minted = v.update(_tb((A("add"), 1)))
                assert (verd, res) == (OK, UPD_OK), (rnd, i)
                cur[i] = _oracle_update(oorset, (A("add"), 1), cur[i], minted)[1]
        for i in range(0, 100, 7):
            assert vs[i].read() == (OK, _tb(cur[i])), i
        # variable 0 binds variable 1's state: 6 tokens on element 1 in variable 0
        st, cur[0] = 1, oorset.merge(cur[0], cur[1])
        assert vs[0].bind(_tb(cur[1])) == (OK, st)
        assert vs[0].read() == (OK, _tb(cur[0]))
        s1 = ctx.nif_stats()
        assert s1["dict_resets"] == s0["dict_resets"]
        assert s1["fallbacks"] == s0["fallbacks"]
        assert s1["vars_spilled"] == s0["vars_spilled"]
        # binds of many variables of different namespaces in one call
        vals = [oorset.merge(cur[i], cur[(i + 1) % 100]) for i in range(100)]
        got = ctx.var_bind_many(list(zip(vs, [_tb(x) for x in vals])))
        for i in range(100):
            want_st = 0 if exact_eq(cur[i], vals[i]) else 1
            assert got[i] == (OK, want_st), i
            cur[i] = vals[i]
        for i in range(0, 100, 9):
            assert vs[i].read() == (OK, _tb(cur[i])), i
        assert ctx.nif_stats()["dict_resets"] == s0["dict_resets"]
        for v in vs:
            v.close()
    finally:
        ctx.close()


def test_replicas_bind_each_others_updates_in_one_pass():
    """Three replicas of one variable in one namespace (laspj_var_create_replica): every
    update mints a token the namespace then knows, so replica B binding replica A's state
    takes one device pass and registers nothing; the converged replicas equal the oracle's
    merge of the three."""
    ctx = _ctx()
    try:
        rng = random.Random(17)
        a = ctx.var("orset")
        reps = [a, a.replica(), a.replica()]
        cur = [[] for _ in reps]
        elems = list(range(40))
        for r, v in enumerate(reps):
            for e in rng.sample(elems, 20):
                verd, res, _e, minted = v.update(_tb((A("add"), e)))
                assert (verd, res) == (OK, UPD_OK)
                cur[r] = _oracle_update(oorset, (A("add"), e), cur[r], minted)[1]
        imgs = [v.read()[1] for v in reps]
        assert imgs == [_tb(c) for c in cur]
        s0 = ctx.nif_stats()
        orig = list(cur)
        for r, v in enumerate(reps):
            for q in range(3):
                if q == r:
                    continue
                want_st = 0 if exact_eq(cur[r], orig[q]) else 1
                assert v.bind(imgs[q]) == (OK, want_st)
                cur[r] = oorset.merge(cur[r], orig[q])
        s1 = ctx.nif_stats()
        assert s1["device_passes"] - s0["device_passes"] == 6
        assert s1["registrations"] == s0["registrations"]
        for v, c in zip(reps, cur):
            assert v.read() == (OK, _tb(c))
        assert exact_eq(cur[0], cur[1]) and exact_eq(cur[1], cur[2])
        # an update on one replica, a remove on another, then a bind each way
        verd, res, _e, minted = reps[0].update(_tb((A("add"), 99)))
        cur[0] = _oracle_update(oorset, (A("add"), 99), cur[0], minted)[1]
        gone = cur[1][0][0]
        assert reps[1].update(_tb((A("remove"), gone)))[:2] == (OK, UPD_OK)
        cur[1] = _oracle_update(oorset, (A("remove"), gone), cur[1], [])[1]
        s2 = ctx.nif_stats()
        assert reps[1].bind(_tb(cur[0])) == (OK, 1)
        assert reps[0].bind(_tb(cur[1])) == (OK, 1)
        assert ctx.nif_stats()["registrations"] == s2["registrations"]
        both = oorset.merge(cur[0], cur[1])
        assert reps[0].read() == (OK, _tb(both)) and reps[1].read() == (OK, _tb(both))
    finally:
        ctx.close()


def test_bind_of_unseen_tokens_redoes_only_failed_segments():
    """A bind whose image carries tokens the variable's namespace has not seen, of a form the
    decoder cannot take on the spot (tuple tokens here; binaries are taken in one pass, see
    below), decodes, registers the failing segments' terms, patches the images and decodes
    again only those segments over the cells the first pass left: two device passes, one
    registration, the oracle's merge.  More failing segments than a redo pass lists, or a
    new element (images rebuilt), take a full second pass — the same answers."""
    from lasp_amd import _lib
    ctx = _ctx()
    try:
        rng = random.Random(23)
        ctx.set_tuning(_lib.TUNE_ETF_SEG, 256)          # many segments per payload
        tok = lambda c, e: (bytes([c]) + e.to_bytes(4, "big") + bytes(15),)   # noqa: E731
        base = [(e, [(tok(1, e), e % 7 == 0)]) for e in range(3000)]
        var = ctx.var("orset")
        assert var.write(_tb(base)) == OK
        cur = base
        for case, nnew, new_elem in (("few", 5, False), ("many", 120, False),
                                     ("element", 3, True)):
            picks = sorted(rng.sample(range(3000), nnew))
            add = {e: (bytes(rng.getrandbits(8) for _ in range(20)),) for e in picks}
            val = [(e, sorted(ts + ([(add[e], False)] if e in add else []), key=_key))
                   for e, ts in cur]
            if new_elem:
                val = sorted(val + [(5000, [((b"\x09" * 20,), False)])], key=lambda x: _key(x[0]))
            s0 = ctx.nif_stats()
            assert var.bind(_tb(val)) == (OK, 1), case
            s1 = ctx.nif_stats()
            cur = oorset.merge(cur, val)
            assert var.read() == (OK, _tb(cur)), case
            assert s1["fallbacks"] == s0["fallbacks"]
            if case == "few":
                assert s1["device_passes"] - s0["device_passes"] == 2
                assert s1["registrations"] - s0["registrations"] == 1
            # binding the same state again: all known, one pass, a no-op
            s2 = ctx.nif_stats()
            assert var.bind(_tb(cur)) == (OK, 0), case
            assert ctx.nif_stats()["device_passes"] - s2["device_passes"] == 1
        ctx.set_tuning(_lib.TUNE_ETF_SEG, 0)
    finally:
        ctx.close()


def test_group_commit_binds_from_many_threads():
    """Sixteen threads binding their own variables through ONE context at once
    (laspj_var_etf_bind's group commit: binds queued while a pass runs share the next
    pass): every answer and every variable's value is the oracle's; the passes are fewer
    than the binds."""
    import threading
    ctx = _ctx()
    try:
        rng = random.Random(31)
        elems = list(range(200))
        nthr, per = 16, 12
        vs = [ctx.var("orset") for _ in range(nthr)]
        vals = [[[(e, [(bytes([t, k]) + e.to_bytes(4, "big") + bytes(14), k % 3 == 0)])
                  for e in sorted(rng.sample(elems, 50))] for k in range(per)]
                for t in range(nthr)]
        got = [[None] * per for _ in range(nthr)]
        errs = []
        go = threading.Barrier(nthr)

        def work(t):
            try:
                go.wait()
                for k in range(per):
                    got[t][k] = vs[t].bind(_tb(vals[t][k]))
            except Exception as e:       # noqa: BLE001
                errs.append(repr(e))

        s0 = ctx.nif_stats()
        ths = [threading.Thread(target=work, args=(t,)) for t in range(nthr)]
        for th in ths:
            th.start()
        for th in ths:
            th.join(timeout=120)
        assert not errs, errs[:3]
        passes = ctx.nif_stats()["device_passes"] - s0["device_passes"]
        for t in range(nthr):
            cur = []
            for k in range(per):
                want_st = 0 if exact_eq(cur, vals[t][k]) else 1
                assert got[t][k] == (OK, want_st), (t, k)
                cur = oorset.merge(cur, vals[t][k])
            assert vs[t].read() == (OK, _tb(cur)), t
        assert passes < nthr * per * 2            # (registration passes included)
    finally:
        ctx.close()


def test_group_commit_waiters_stage_large_payloads():
    """Group commit with payloads past the waiters' staging threshold (64 KiB): the waiting
    threads copy their own payloads into pinned blocks and the leader's pass gathers them
    on the device at byte offsets of every alignment (payload lengths vary by a few bytes)
    — every answer and every value is the oracle's."""
    import threading
    ctx = _ctx()
    try:
        rng = random.Random(47)
        elems = list(range(6000))
        nthr, per = 8, 6
        vs = [ctx.var("orset") for _ in range(nthr)]
        # token images of one length (the device decoder's), element counts varied so the
        # images' lengths (and so the gather's byte offsets) fall on every residue mod 16
        vals = [[[(e, [(bytes([t, k]) + e.to_bytes(4, "big") + bytes(14), (e + k) % 3 == 0)])
                  for e in sorted(rng.sample(elems, 2200 + 7 * t + k))] for k in range(per)]
                for t in range(nthr)]
        assert all(len(_tb(v)) >= 64 << 10 for row in vals for v in row)
        got = [[None] * per for _ in range(nthr)]
        errs = []
        go = threading.Barrier(nthr)

        def work(t):
            try:
                go.wait()
                for k in range(per):
                    got[t][k] = vs[t].bind(_tb(vals[t][k]))
            except Exception as e:       # noqa: BLE001
                errs.append(repr(e))

        ths = [threading.Thread(target=work, args=(t,)) for t in range(nthr)]
        for th in ths:
            th.start()
        for th in ths:
            th.join(timeout=120)
        assert not errs, errs[:3]
        for t in range(nthr):
            cur = []
            for k in range(per):
                want_st = 0 if exact_eq(cur, vals[t][k]) else 1
                assert got[t][k] == (OK, want_st), (t, k)
                cur = oorset.merge(cur, vals[t][k])
            assert vs[t].read() == (OK, _tb(cur)), t
    finally:
        ctx.close()


def test_bind_many_fresh_namespaces():
    """One bind_many over sixteen fresh variables (sixteen namespaces with no dictionary
    yet, registered in the call, decoded in one launch), then again with new tokens and
    repeats: statuses and values are the oracle's."""
    ctx = _ctx()
    try:
        rng = random.Random(32)
        vs = [ctx.var("orset") for _ in range(16)]
        cur = [[] for _ in vs]
        for rnd in range(4):
            vals = [[(e, [(bytes([t, rnd]) + e.to_bytes(4, "big") + bytes(14), rnd % 2 == 1)])
                     for e in sorted(rng.sample(range(200), 50))] for t in range(16)]
            if rnd == 3:
                vals[4] = cur[4]
            got = ctx.var_bind_many(list(zip(vs, [_tb(v) for v in vals])))
            for t in range(16):
                want = 0 if exact_eq(cur[t], vals[t]) else 1
                assert got[t] == (OK, want), (rnd, t)
                cur[t] = oorset.merge(cur[t], vals[t])
                assert vs[t].read() == (OK, _tb(cur[t])), (rnd, t)
    finally:
        ctx.close()


def test_wide_namespace_element_past_64_tokens():
    """The reference mints a token per add and never collects them (lasp_orset.erl:222-241,
    261-262): an element past 64 tokens widens its namespace's cells to k {p, r} pairs
    (token slot t in pair t / 64) instead of handing the variable back to Erlang.  Three
    replicas add element 1 200 times between them, bind each other's states, remove it,
    and answer value/1, threshold and read as the oracle does; write/4 and bind_many of wide
    images, and image calls whose operands carry 100 tokens on an element, agree too."""
    ctx = _ctx()
    try:
        rng = random.Random(41)
        a = ctx.var("orset")
        reps = [a, a.replica(), a.replica()]
        cur = [[] for _ in reps]
        for k in range(240):
            r = k % 3
            op = (A("add"), 1) if k % 6 else (A("add"), rng.randrange(8))
            verd, res, _e, minted = reps[r].update(_tb(op))
            assert (verd, res) == (OK, UPD_OK), k
            cur[r] = _oracle_update(oorset, op, cur[r], minted)[1]
            if k % 40 == 39:
                assert reps[r].read() == (OK, _tb(cur[r])), k
        assert ctx.nif_stats()["fallbacks"] == 0
        imgs = [v.read()[1] for v in reps]
        assert imgs == [_tb(c) for c in cur]
        orig = list(cur)
        for r, v in enumerate(reps):
            for q in range(3):
                if q != r:
                    assert v.bind(imgs[q]) == (OK, 0 if exact_eq(cur[r], orig[q]) else 1)
                    cur[r] = oorset.merge(cur[r], orig[q])
        assert all(v.read() == (OK, _tb(c)) for v, c in zip(reps, cur))
        ones = [ts for e, ts in cur[0] if e == 1][0]
        assert len(ones) > 150
        th = orig[1]
        assert reps[0].threshold(_tb(th)) == (OK, olat.threshold_met("lasp_orset", cur[0], th))
        assert reps[0].value() == (OK, _tb(oorset.value(cur[0])))
        assert reps[2].update(_tb((A("remove"), 1)))[:2] == (OK, UPD_OK)
        cur[2] = _oracle_update(oorset, (A("remove"), 1), cur[2], [])[1]
        assert reps[2].read() == (OK, _tb(cur[2]))
        assert reps[2].value() == (OK, _tb(oorset.value(cur[2])))
        assert reps[0].bind(_tb(cur[2])) == (OK, 1)
        cur[0] = oorset.merge(cur[0], cur[2])
        assert reps[0].read() == (OK, _tb(cur[0]))
        # write/4 of a wide image into a fresh variable, bind_many beside a narrow one
        w = ctx.var("orset")
        assert w.write(_tb(cur[1])) == OK and w.resident
        n = ctx.var("orset")
        small = [(3, [(b"\x05" * 20, False)])]
        got = ctx.var_bind_many([(w, _tb(cur[0])), (n, _tb(small))])
        assert got == [(OK, 0 if exact_eq(cur[1], oorset.merge(cur[1], cur[0])) else 1), (OK, 1)]
        assert w.read() == (OK, _tb(oorset.merge(cur[1], cur[0])))
        assert n.read() == (OK, _tb(small))
        # image calls: operands of 100 tokens on an element, then narrow ones again
        toks = sorted(bytes(rng.getrandbits(8) for _ in range(20)) for _ in range(200))
        x = [(1, [(t, i % 4 == 0) for i, t in enumerate(toks[:100])]), (2, [(toks[150], False)])]
        y = [(1, [(t, i % 5 == 0) for i, t in enumerate(toks[50:150])])]
        assert ctx.nif_merge(_tb(x), _tb(y)) == (OK, _tb(oorset.merge(x, y)))
        assert ctx.nif_merge(_tb(y), _tb(x)) == (OK, _tb(oorset.merge(y, x)))
        assert ctx.nif_value(_tb(x)) == (OK, _tb(oorset.value(x)))
        assert ctx.nif_equal(_tb(x), _tb(x)) == (OK, True)
        assert ctx.nif_inflation(_tb(y), _tb(oorset.merge(x, y))) == (OK, True)
        z = [(1, [(toks[199], False)]), (4, [(toks[198], True)])]
        assert ctx.nif_merge(_tb(z), _tb(small)) == (OK, _tb(oorset.merge(z, small)))
        assert ctx.nif_stats()["fallbacks"] == 0
    finally:
        ctx.close()


def test_bind_takes_unseen_binary_tokens_in_one_pass():
    """Another node's update mints a 20-byte binary token (lasp_orset.erl:222-230, 261-262):
    a bind of its state decodes the unseen tokens of known elements on the device in one
    pass (each gets its element's next free slot; the host dictionary registers them after
    the call), whether they sort before, between or after the known ones, several on one
    element, two between the same neighbours; the answers, the values read back, value/1
    and threshold agree with the oracle, and binding the same state again is a one-pass
    no-op.  An element pushed past 64 tokens this way takes the two-pass path and widens."""
    from lasp_amd import _lib
    for seg in (0, 256):
        ctx = _ctx()
        try:
            rng = random.Random(29 + seg)
            if seg:
                ctx.set_tuning(_lib.TUNE_ETF_SEG, seg)
            mid = lambda b: bytes([b]) + bytes(rng.getrandbits(8) for _ in range(19))  # noqa: E731
            base = [(e, sorted([(mid(0x40 + 2 * k), k % 2 == 0) for k in range(3)], key=_key))
                    for e in range(2000)]
            var = ctx.var("orset")
            assert var.write(_tb(base)) == OK
            cur = base
            for rnd in range(6):
                val = []
                picks = set(rng.sample(range(2000), 40))
                for e, ts in cur:
                    ts = list(ts)
                    if e in picks:
                        # before the first known, between two, after the last, two between
                        # the same neighbours, several at once
                        kind = rng.randrange(5)
                        if kind == 0:
                            new = [b"\x00" + bytes(rng.getrandbits(8) for _ in range(19))]
                        elif kind == 1:
                            new = [mid(0x41)]
                        elif kind == 2:
                            new = [b"\xff" + bytes(rng.getrandbits(8) for _ in range(19))]
                        elif kind == 3:
                            new = [mid(0x43), mid(0x43)]
                        else:
                            new = [mid(rng.randrange(256)) for _ in range(3)]
                        ts += [(t, rng.random() < 0.3) for t in new]
                    val.append((e, sorted(ts, key=_key)))
                s0 = ctx.nif_stats()
                assert var.bind(_tb(val)) == (OK, 1), (seg, rnd)
                s1 = ctx.nif_stats()
                cur = oorset.merge(cur, val)
                assert s1["device_passes"] - s0["device_passes"] == 1, (seg, rnd)
                assert s1["device_new_tokens"] - s0["device_new_tokens"] >= 40, (seg, rnd)
                assert s1["fallbacks"] == s0["fallbacks"]
                assert var.read() == (OK, _tb(cur)), (seg, rnd)
                s2 = ctx.nif_stats()
                assert var.bind(_tb(val)) == (OK, 0)
                assert ctx.nif_stats()["device_passes"] - s2["device_passes"] == 1
            assert var.value() == (OK, _tb(oorset.value(cur)))
            assert var.threshold(_tb(base)) == (OK, olat.threshold_met("lasp_orset", cur, base))
            # a threshold and a value/1 operand carrying unseen tokens: one pass each
            th = oorset.merge(cur, [(3, [(b"\x01" * 20, False)]), (4, [(b"\xfe" * 20, True)])])
            s0 = ctx.nif_stats()
            assert var.threshold(_tb(th)) == (OK, olat.threshold_met("lasp_orset", cur, th))
            assert var.threshold(_tb(cur)) == (OK, True)
            vimg = oorset.merge(cur, [(5, [(b"\x02" * 20, False)]), (6, [(b"\xfd" * 20, True)])])
            assert ctx.nif_value(_tb(vimg)) == (OK, _tb(oorset.value(vimg)))
            s1 = ctx.nif_stats()
            assert s1["device_passes"] - s0["device_passes"] <= 4
            assert s1["device_new_tokens"] > s0["device_new_tokens"]
            # element 7 past 64 tokens: two passes, the namespace widens, the oracle's answer
            e7 = [ts for e, ts in cur if e == 7][0]
            more = [(e, sorted(ts + ([(mid(rng.randrange(256)), False) for _ in range(70)]
                                     if e == 7 else []), key=_key)) for e, ts in cur]
            assert len(e7) + 70 > 64
            assert var.bind(_tb(more)) == (OK, 1)
            cur = oorset.merge(cur, more)
            assert var.read() == (OK, _tb(cur))
            assert ctx.nif_stats()["namespaces_widened"] == 1
        finally:
            ctx.close()


def test_tokens_no_bucket_window_separates():
    """Tokens of one element that no single 10-bit window of their records tells apart
    (b"A" + x, b"B" + x, b"A" + y: the first pair differs in one byte, the last pair only
    where the first pair agrees): that element is matched template by template while
    every other element keeps its bucket table — the dictionary stays patchable, binds
    decode in one pass and an update patches instead of rebuilding."""
    ctx = _ctx()
    try:
        rng = random.Random(43)
        x, y = bytes(19), bytes([7]) * 19
        bad = [(b"A" + x, False), (b"A" + y, True), (b"B" + x, False)]
        base = [(e, [(bytes([0x30 + k]) + bytes(rng.getrandbits(8) for _ in range(19)),
                      k == 1) for k in range(2)]) for e in range(3000)]
        base[1234] = (1234, sorted(bad, key=_key))
        var = ctx.var("orset")
        assert var.write(_tb(base)) == OK
        assert var.read() == (OK, _tb(base))
        cur = base
        s0 = ctx.nif_stats()
        for k in range(6):
            op = (A("add"), 1234 if k % 3 == 1 else rng.randrange(3000))
            verd, res, _e, minted = var.update(_tb(op))
            assert (verd, res) == (OK, UPD_OK)
            cur = _oracle_update(oorset, op, cur, minted)[1]
        s1 = ctx.nif_stats()
        assert s1["image_rebuilds"] == s0["image_rebuilds"]
        assert var.read() == (OK, _tb(cur))
        other = [(e, sorted(ts + ([(b"Z" + bytes(rng.getrandbits(8) for _ in range(19)), False)]
                                  if e % 30 == 4 or e == 1234 else []), key=_key))
                 for e, ts in cur]
        s2 = ctx.nif_stats()
        assert var.bind(_tb(other)) == (OK, 1)
        assert ctx.nif_stats()["device_passes"] - s2["device_passes"] == 1
        cur = oorset.merge(cur, other)
        assert var.read() == (OK, _tb(cur))
        assert var.value() == (OK, _tb(oorset.value(cur)))
        assert ctx.nif_merge(_tb(base), _tb(cur)) == (OK, _tb(oorset.merge(base, cur)))
    finally:
        ctx.close()


def test_new_token_decode_fuzz():
    """The one-pass new-token decode against the oracle on random binds: unseen binary
    tokens anywhere in an element (several per element, runs of them), mixed with
    non-canonical states — two tokens swapped (descending), a token twice, a token of
    another length — which must answer FALLBACK and leave the variable as it was (the
    reference's own clause then runs), exactly as the two-pass path would."""
    for soak in range(SOAK):
        _new_token_fuzz_round(97 + 1000 * soak)


def _new_token_fuzz_round(seed):
    ctx = _ctx()
    try:
        rng = random.Random(seed)
        tok = lambda: bytes(rng.getrandbits(8) for _ in range(20))  # noqa: E731
        base = [(e, sorted([(tok(), rng.random() < 0.3) for _ in range(rng.randint(1, 3))],
                           key=_key)) for e in range(600)]
        var = ctx.var("orset")
        assert var.write(_tb(base)) == OK
        cur = base
        kinds = {"ok": 0, "swap": 0, "twice": 0, "length": 0}
        for it in range(80):
            val = []
            bad = rng.choice(["ok"] * 5 + ["swap", "twice", "length"])
            victim = rng.randrange(600)
            for e, ts in cur:
                ts = list(ts)
                if rng.random() < 0.08 or e == victim:
                    ts += [(tok(), rng.random() < 0.3) for _ in range(rng.randint(1, 4))]
                ts = sorted(ts, key=_key)
                if e == victim and bad == "swap" and len(ts) >= 2:
                    ts[0], ts[1] = ts[1], ts[0]
                elif e == victim and bad == "twice":
                    ts = sorted(ts + [ts[0]], key=_key)
                elif e == victim and bad == "length":
                    ts = sorted(ts + [(tok() + b"x", False)], key=_key)
                if len(ts) > 60:
                    ts = ts[:60]
                val.append((e, ts))
            kinds[bad] += 1
            got = var.bind(_tb(val))
            if bad in ("swap", "twice"):
                assert got[0] == FALLBACK, (it, bad)
                assert var.read() == (OK, _tb(cur)), (it, bad)
                continue
            assert got[0] == OK, (it, bad)
            st, new = 0 if exact_eq(cur, oorset.merge(cur, val)) else 1, oorset.merge(cur, val)
            assert got == (OK, st), (it, bad)
            cur = new
            if it % 5 == 0 or bad == "length":
                got_img = var.read()
                if got_img != (OK, _tb(cur)):
                    g = oetf.binary_to_term(got_img[1])
                    diff = [(a, b) for a, b in zip(g, cur) if not exact_eq(a, b)][:2]
                    raise AssertionError((seed, it, bad, len(g), len(cur),
                                          [(a[0], len(a[1]), b[0], len(b[1])) for a, b in diff],
                                          ctx.nif_stats()))
        assert var.read() == (OK, _tb(cur))
        assert min(kinds.values()) > 0
        assert ctx.nif_stats()["device_new_tokens"] > 0 or kinds["length"] > 0
    finally:
        ctx.close()


def test_var_union_matches_oracle():
    """lasp_core:union/7's body re-run over resident variables of one namespace
    (laspj_var_union): out := merge(out, orddict:merge(keep-left, l, r)), the status the
    bind's `Value0 =:= AccValue` test gives — over random updates of l and r (adds,
    removes, new elements), against the oracle's union body and bind; out may be l; a
    wide namespace too; G-Sets and variables of two namespaces answer FALLBACK."""
    from oracle import core as ocore
    ctx = _ctx()
    try:
        rng = random.Random(53)
        for wide in (False, True):
            l = ctx.var("orset")
            r, out = l.replica(), l.replica()
            cur = {"l": [], "r": [], "out": []}
            vs = {"l": l, "r": r}
            for it in range(40):
                name = rng.choice(("l", "r"))
                e = rng.randrange(40)
                if wide and it < 4:
                    ops = [(A("add_all"), [e] * 1)] + [(A("add"), 7)] * 30
                else:
                    ops = [(A("add"), e) if rng.random() < 0.7 else (A("remove"), e)]
                for op in ops:
                    verd, res, _e, minted = vs[name].update(_tb(op))
                    assert verd == OK
                    want = _oracle_update(oorset, op, cur[name], minted)
                    if want[0] == "ok":
                        cur[name] = want[1]
                acc = ocore.union_body("lasp_orset", cur["l"], cur["r"])
                st = 0 if exact_eq(cur["out"], acc) else 1
                assert out.union(l, r) == (OK, st), (wide, it)
                if st:
                    cur["out"] = oorset.merge(cur["out"], acc)
                assert out.read() == (OK, _tb(cur["out"])), (wide, it)
            # out may be one of its operands
            acc = ocore.union_body("lasp_orset", cur["l"], cur["r"])
            st = 0 if exact_eq(cur["l"], acc) else 1
            assert l.union(l, r) == (OK, st)
            cur["l"] = oorset.merge(cur["l"], acc) if st else cur["l"]
            assert l.read() == (OK, _tb(cur["l"]))
            if wide:
                assert ctx.nif_stats()["namespaces_widened"] >= 1
        other = ctx.var("orset")
        assert other.union(l, r)[0] == FALLBACK
        g1 = ctx.var("gset")
        g2 = g1.replica()
        assert g1.union(g1, g2)[0] == FALLBACK
    finally:
        ctx.close()


def test_group_commit_wide_and_new_tokens_together():
    """Eight threads binding through one context at once, each into its own variable, half
    of them in a namespace widened by a hot element (host-encoded operands), every image
    carrying tokens the namespace has not seen (another node's updates): the group commit
    mixes wide and narrow namespaces, one-pass new tokens and two-pass registrations in
    one batch — every answer and value is the oracle's."""
    import threading
    ctx = _ctx()
    try:
        rng = random.Random(59)
        nthr, per = 8, 6
        vs, cur = [], []
        for t in range(nthr):
            v = ctx.var("orset")
            base = [(e, [(bytes([t, e]) + bytes(18), False)]) for e in range(200)]
            assert v.write(_tb(base)) == OK
            if t % 2:
                for _ in range(70):                      # a hot element: the namespace widens
                    verd, res, _e, minted = v.update(_tb((A("add"), 5)))
                    assert (verd, res) == (OK, UPD_OK)
                    base = _oracle_update(oorset, (A("add"), 5), base, minted)[1]
            vs.append(v)
            cur.append(base)
        vals = [[None] * per for _ in range(nthr)]
        for t in range(nthr):
            c = cur[t]
            for k in range(per):
                c = [(e, sorted(ts + ([(bytes(rng.getrandbits(8) for _ in range(20)), False)]
                                      if rng.random() < 0.1 else []), key=_key)) for e, ts in c]
                if k == 3:
                    c = sorted(c + [(1000 + t, [(bytes([9, t]) + bytes(18), True)])],
                               key=lambda x: _key(x[0]))
                vals[t][k] = c
        got = [[None] * per for _ in range(nthr)]
        errs = []
        go = threading.Barrier(nthr)

        def work(t):
            try:
                go.wait()
                for k in range(per):
                    got[t][k] = vs[t].bind(_tb(vals[t][k]))
            except Exception as e:       # noqa: BLE001
                errs.append(repr(e))

        ths = [threading.Thread(target=work, args=(t,)) for t in range(nthr)]
        for th in ths:
            th.start()
        for th in ths:
            th.join(timeout=120)
        assert not errs, errs[:3]
        for t in range(nthr):
            c = cur[t]
            for k in range(per):
                want = 0 if exact_eq(c, vals[t][k]) else 1
                assert got[t][k] == (OK, want), (t, k)
                c = oorset.merge(c, vals[t][k])
            assert vs[t].read() == (OK, _tb(c)), t
        assert ctx.nif_stats()["namespaces_widened"] >= nthr // 2
    finally:
        ctx.close()
