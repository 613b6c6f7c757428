"""crdt_statem_eqc:prop_converge (test/crdt_statem_eqc.erl:94-106) with hypothesis.

Commands create / update(gen_op) / merge(A, B) / crdt_equals(A, B) run over simulated
replicas; merge(A, B) must equal merge(B, A) (:158-160), and the fold-merge of all
replicas (:134-140) must have the value the model predicts.  The model is the
reference's own EQC model: lasp_orset.erl:305-382 (adds tagged with a counter, removes
observe the local adds) and lasp_gset.erl:171-195.  gen_op follows
lasp_orset.erl:294-303 / lasp_gset.erl:167-169.

CPU: the oracle restatement.  GPU: the device mirrors (lasp_amd.orset / lasp_amd.gset).
"""

import os

import pytest
from hypothesis import HealthCheck, given, settings, strategies as st

from oracle import gset as ogset, orset as oorset
from oracle.terms import Key

SOAK = int(__import__("os").environ.get("LASPJ_SOAK", "1"))   # x examples for a soak run

ELEM = st.integers(min_value=-3, max_value=6)
GEN_UPDATE = st.one_of(
    st.tuples(st.just("add"), ELEM), st.tuples(st.just("remove"), ELEM),
    st.tuples(st.just("add_all"), st.lists(ELEM, max_size=4)),
    st.tuples(st.just("remove_all"), st.lists(ELEM, max_size=4)))
GEN_OP = st.one_of(GEN_UPDATE, st.tuples(st.just("update"), st.lists(GEN_UPDATE, min_size=1, max_size=4)))
GSET_OP = st.one_of(st.tuples(st.just("add"), ELEM),
                    st.tuples(st.just("add_all"), st.lists(ELEM, min_size=1, max_size=4)))


def commands(op):
    cmd = st.one_of(
        st.tuples(st.just("create")),
        st.tuples(st.just("update"), op, st.integers(0, 7)),
        st.tuples(st.just("merge"), st.integers(0, 7), st.integers(0, 7)),
        st.tuples(st.just("equals"), st.integers(0, 7), st.integers(0, 7)))
    return st.lists(cmd, max_size=25)


# ------------------------------------------------------------------ models

class ORSetModel:
    """lasp_orset.erl:305-382."""

    def __init__(self):
        self.cnt = 0
        self.d = {}

    def create(self, i):
        self.d[i] = (frozenset(), frozenset())

    def apply(self, i, op):
        self.cnt, self.d = self._upd(i, op, (self.cnt, dict(self.d)))

    def _upd(self, i, op, state):
        cnt, d = state
        kind = op[0]
        if kind == "update":
            return self._do_updates(i, op[1], state, state)
        if kind == "add":
            a, r = d[i]
            d = dict(d)
            d[i] = (a | {(op[1], cnt + 1)}, r)
            return (cnt + 1, d)
        if kind == "remove":
            a, r = d[i]
            d = dict(d)
            d[i] = (a, r | {(e, x) for (e, x) in a if e == op[1]})
            return (cnt, d)
        if kind == "add_all":
            for e in op[1]:
                state = self._upd(i, ("add", e), state)
            return state
        if kind == "remove_all":
            a, r = d[i]
            members = {e for e, _ in a | r}
            if set(op[1]) <= members:
                for e in op[1]:
                    state = self._upd(i, ("remove", e), state)
            return state
        raise ValueError(op)

    def _do_updates(self, i, ups, old, new):
        for up in ups:
            if up[0] in ("add_all", "remove_all") and up[1] == []:
                continue
            nn = self._upd(i, up, new)
            if up[0] in ("remove", "remove_all") and nn[1] == new[1] and nn[0] == new[0]:
                removed = [e for e, _ in new[1][i][1]]
                arg = up[1]
                ok = (set(arg) <= set(removed) and removed != []) if isinstance(arg, list) \
                    else arg in removed
                if not ok:
                    return old
                continue
            new = nn
        return new

    def merge(self, src, dst):
        fa, fr = self.d[dst]
        ta, tr = self.d[src]
        self.d[dst] = (fa | ta, fr | tr)

    def value(self):
        a, r = set(), set()
        for x, y in self.d.values():
            a |= x
            r |= y
        return sorted({e for e, _ in a - r})


class GSetModel:
    """lasp_gset.erl:171-195."""

    def __init__(self):
        self.d = {}

    def create(self, i):
        self.d[i] = frozenset()

    def apply(self, i, op):
        add = {op[1]} if op[0] == "add" else set(op[1])
        self.d[i] = self.d[i] | add

    def merge(self, src, dst):
        self.d[dst] = self.d[dst] | self.d[src]

    def value(self):
        out = set()
        for v in self.d.values():
            out |= v
        return sorted(out)


# ------------------------------------------------------------------ runner

def run(cmds, mod, model, equal, merge, update, new, value):
    vnodes = []       # [(id, crdt)]
    nid = 0
    for c in cmds:
        if c[0] == "create":
            vnodes.append((nid, new()))
            model.create(nid)
            nid += 1
        elif not vnodes:
            continue
        elif c[0] == "update":
            k = c[2] % len(vnodes)
            vid, crdt = vnodes[k]
            res = update(c[1], vid, crdt)
            if res[0] == "ok":
                vnodes[k] = (vid, res[1])
            model.apply(vid, c[1])
        elif c[0] == "merge":
            s, d = vnodes[c[1] % len(vnodes)], vnodes[c[2] % len(vnodes)]
            k = c[2] % len(vnodes)
            vnodes[k] = (d[0], merge(s[1], d[1]))
            model.merge(s[0], d[0])
        elif c[0] == "equals":
            a, b = vnodes[c[1] % len(vnodes)][1], vnodes[c[2] % len(vnodes)][1]
            assert equal(merge(a, b), merge(b, a))          # crdt_statem_eqc.erl:158-160
    if vnodes:
        merged = vnodes[0][1]
        for _, c in vnodes[1:]:
            merged = merge(c, merged)                        # merge_crdts/2 :134-140
    else:
        merged = new()
    got = sorted(value(merged), key=Key)
    assert got == model.value()


SETTINGS = settings(max_examples=300 * SOAK, deadline=None,
                    suppress_health_check=[HealthCheck.too_slow])


@SETTINGS
@given(commands(GEN_OP))
def test_orset_converges(cmds):
    run(cmds, "lasp_orset", ORSetModel(), oorset.equal, oorset.merge,
        lambda op, a, s: oorset.update(op, a, s), oorset.new, oorset.value)


@SETTINGS
@given(commands(GSET_OP))
def test_gset_converges(cmds):
    run(cmds, "lasp_gset", GSetModel(), ogset.equal, ogset.merge,
        lambda op, a, s: ogset.update(op, a, s), ogset.new, ogset.value)


@pytest.mark.gpu
@settings(max_examples=60 * int(os.environ.get("LASPJ_SOAK", "1")), deadline=None, suppress_health_check=[HealthCheck.too_slow])
@given(commands(GEN_OP))
def test_gpu_orset_converges(cmds):
    from lasp_amd import orset as do
    run(cmds, "lasp_orset", ORSetModel(), do.equal, do.merge,
        lambda op, a, s: do.update(op, a, s), do.new, do.value)


@pytest.mark.gpu
@settings(max_examples=40 * int(os.environ.get("LASPJ_SOAK", "1")), deadline=None, suppress_health_check=[HealthCheck.too_slow])
@given(commands(GSET_OP))
def test_gpu_gset_converges(cmds):
    from lasp_amd import gset as dg
    run(cmds, "lasp_gset", GSetModel(), dg.equal, dg.merge,
        lambda op, a, s: dg.update(op, a, s), dg.new, dg.value)
