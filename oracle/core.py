"""lasp_core restatement: bind / update / read and the monotonic combinators —
oracle (TEST INFRASTRUCTURE).

The combinator *bodies* (`*_body`) restate the `Function(Scope)` closures of
src/lasp_core.erl:460-712 exactly, including their list-level behaviour (`Acc ++ ...`
order, duplicates, keep-left union, descending product tokens).  `Store` restates
declare / bind / update / read (lasp_core.erl:197-364, 839-844) over one in-memory
store — the ETS-backend single-node path the EQC harness uses (test/lasp_eqc.erl,
include/lasp.hrl:19-23) — and replaces the asynchronous `lasp_process` loop
(src/lasp_process.erl:61-95) with a synchronous equivalent: after every write, each
combinator whose input is now a strict inflation of the value it last saw re-reads it
and re-runs its body.
"""

from __future__ import annotations

from . import otp, orset, orset_gbtree, gset, lattice
from .terms import exact_eq

# ----------------------------------------------------------------------------- types

_TYPES = {}


class _GCounter:
    """riak_dt_gcounter subset used by threshold reads (lasp_lattice.erl:87-90):
    orddict Actor -> Count; merge is the per-actor max."""

    @staticmethod
    def new():
        return []

    @staticmethod
    def value(c):
        return sum(n for _a, n in c)

    @staticmethod
    def update(op, actor, c, tokens=None):
        # riak_dt_gcounter:update(increment | {increment, N}, Actor, C): orddict
        # update_counter(Actor, N, C)
        if op == "increment":
            op = ("increment", 1)
        if isinstance(op, tuple) and len(op) == 2 and op[0] == "increment" and \
                isinstance(op[1], int) and not isinstance(op[1], bool) and op[1] > 0:
            found = otp.orddict_find(actor, c)
            n = 0 if found is None else found[1]
            return ("ok", otp.orddict_store(actor, n + op[1], c))
        raise ValueError(op)

    @staticmethod
    def equal(a, b):
        from .terms import eq
        return eq(list(a), list(b))

    @staticmethod
    def merge(a, b):
        return otp.orddict_merge(lambda _k, x, y: max(x, y), a, b)


class _ORSet:
    new = staticmethod(orset.new)
    value = staticmethod(orset.value)
    merge = staticmethod(orset.merge)

    @staticmethod
    def update(op, actor, s, tokens=None):
        return orset.update(op, actor, s, tokens)


class _GSet:
    new = staticmethod(gset.new)
    value = staticmethod(gset.value)
    merge = staticmethod(gset.merge)

    @staticmethod
    def update(op, actor, s, tokens=None):
        return gset.update(op, actor, s)


class _ORSetGBTree:
    new = staticmethod(orset_gbtree.new)
    value = staticmethod(orset_gbtree.value)
    merge = staticmethod(orset_gbtree.merge)

    @staticmethod
    def update(op, actor, s, tokens=None):
        return orset_gbtree.update(op, actor, s, tokens)


_TYPES["lasp_orset"] = _ORSet
_TYPES["lasp_orset_gbtree"] = _ORSetGBTree
_TYPES["lasp_gset"] = _GSet
_TYPES["riak_dt_gcounter"] = _GCounter


def type_mod(t):
    return _TYPES[t]


# ----------------------------------------------------------------------------- bodies


def union_body(type_, lvalue, rvalue):
    """union/7 body — lasp_core.erl:602-627.  None stands for `undefined`."""
    if lvalue is None or rvalue is None:
        return None
    if type_ == "lasp_orset":
        return otp.orddict_merge(lambda _k, l, _r: l, lvalue, rvalue)
    if type_ == "lasp_gset":
        return list(lvalue) + list(rvalue)
    raise ValueError(type_)


def _entry(element):
    """The bodies' `case Element of {X, Causality} -> ...; X -> ... end`: any 2-tuple
    takes the first (OR-Set) branch, whatever the type (lasp_core.erl:467-474,
    513-521, 560-576, 648-655, 688-695)."""
    if isinstance(element, tuple) and len(element) == 2:
        return element
    return None


def _append(acc, values):
    """`Acc ++ Values`: Values must be a proper list here (an improper result is not a
    Lasp value; the oracle treats it as the crash it becomes at the next merge)."""
    if not isinstance(values, list):
        raise TypeError("badarg: ++ with a non-list")
    return acc + values


def intersection_body(type_, lvalue, rvalue):
    """intersection/7 body — lasp_core.erl:546-589."""
    if lvalue is None or rvalue is None:
        return None
    acc = []
    for element in lvalue:
        e = _entry(element)
        if e is not None:
            x, xc = e
            found = otp.lists_keyfind(x, rvalue)
            if found is False:
                vals = []
            else:
                if not isinstance(xc, list):
                    raise TypeError("badarg: ++ on a non-list")
                vals = [(x, lattice.orset_causal_union(xc, _append([], found[1])))]
        else:
            vals = [element] if otp.lists_member(element, rvalue) else []
        acc = acc + vals
    return acc


def product_body(type_, lvalue, rvalue):
    """product/7 body — lasp_core.erl:499-533 (X-major).  The OR-Set branch's generator
    `{Y, YCausality} <- RValue` skips elements of R that are not 2-tuples."""
    if lvalue is None or rvalue is None:
        return None
    acc = []
    for element in lvalue:
        e = _entry(element)
        if e is not None:
            x, xc = e
            if not isinstance(xc, list):
                raise TypeError("function_clause: lists:foldl on a non-list")
            vals = [((x, y), lattice.orset_causal_product(xc, yc))
                    for y, yc in (t for t in rvalue if _entry(t) is not None)]
        else:
            vals = [(element, y) for y in rvalue]
        acc = acc + vals
    return acc


def map_body(type_, fun, value):
    """map/6 body — lasp_core.erl:641-667."""
    acc = []
    for element in value:
        e = _entry(element)
        acc = acc + [(fun(e[0]), e[1]) if e is not None else fun(element)]
    return acc


def filter_body(type_, fun, value):
    """filter/6 body — lasp_core.erl:681-712 (keeps tombstoned OR-Set elements)."""
    acc = []
    for element in value:
        e = _entry(element)
        v = e[0] if e is not None else element
        if fun(v) is True:
            acc = acc + [element]
    return acc


def fold_body(type_, fun, value):
    """fold/6 body — lasp_core.erl:460-486."""
    acc = []
    for element in value:
        e = _entry(element)
        if e is not None:
            x, c = e
            vals = fun(x)
            if not isinstance(vals, list):
                raise TypeError("bad generator: a list comprehension over a non-list")
            vals = [(v, c) for v in vals]
        else:
            vals = fun(element)
        acc = _append(acc, vals)
    return acc


# ----------------------------------------------------------------------------- store


class Store:
    """Single-store lasp_core (declare / update / bind / read + combinator processes)."""

    def __init__(self, tokens=None):
        self.vars = {}        # id -> {"type", "value", "waiting"}
        self.procs = []       # combinator processes
        self.tokens = tokens or orset.TokenSource(0)
        self._next_id = 0
        self._depth = 0

    # lasp_core.erl:197-218
    def declare(self, type_, id_=None):
        if id_ is None:
            self._next_id += 1
            id_ = f"var{self._next_id}"
        if id_ not in self.vars:
            self.vars[id_] = {"type": type_, "value": type_mod(type_).new(), "waiting": []}
        return ("ok", id_)

    # lasp_core.erl:283-287
    def update(self, id_, op, actor):
        dv = self.vars[id_]
        res = type_mod(dv["type"]).update(op, actor, dv["value"], self.tokens)
        if res[0] != "ok":
            raise RuntimeError(f"badmatch: {res!r}")
        return self.bind(id_, res[1])

    # lasp_core.erl:291-312
    def bind(self, id_, value):
        dv = self.vars[id_]
        t, value0 = dv["type"], dv["value"]
        if exact_eq(_canon(value0), _canon(value)):
            return ("ok", (id_, t, value))
        try:
            merged = type_mod(t).merge(value0, value)
            if _is_inflation(t, value0, merged):
                self._write(t, merged, id_)
        except Exception:       # merge may throw for invalid types (:298, :308-311)
            pass
        return ("ok", (id_, t, value))

    # lasp_core.erl:331-364 (without blocking: returns None and records the waiter)
    def read(self, id_, threshold=("strict", None)):
        dv = self.vars[id_]
        t = dv["type"]
        threshold = _normalise_threshold(t, threshold)
        if lattice.threshold_met(t, dv["value"], threshold):
            return ("ok", (id_, t, dv["value"]))
        dv["waiting"].append(threshold)
        return None

    def value(self, id_):
        return self.vars[id_]["value"]

    # lasp_core.erl:839-844; the waiters' re-check (reply_to_all :765-825) is folded
    # into _propagate, which re-runs the combinator processes.
    def _write(self, t, value, id_):
        dv = self.vars[id_]
        dv["waiting"] = [th for th in dv["waiting"] if not lattice.threshold_met(t, value, th)]
        dv["value"] = value
        self._propagate()

    # ------------------------------------------------------------------ processes
    def _start(self, inputs, body):
        proc = {"inputs": list(inputs), "seen": {i: None for i in inputs}, "body": body}
        self.procs.append(proc)
        self._propagate()
        return ("ok", proc)

    def _propagate(self):
        # lasp_process.erl:61-95, synchronously: while some input strictly inflates the
        # last value a process saw, record it and re-run Function(Scope).
        self._depth += 1
        if self._depth > 1:
            self._depth -= 1
            return
        try:
            changed = True
            while changed:
                changed = False
                for proc in list(self.procs):
                    for i in proc["inputs"]:
                        dv = self.vars[i]
                        last = proc["seen"][i]
                        th = ("strict", type_mod(dv["type"]).new() if last is None else last)
                        if proc not in self.procs:
                            break
                        if last is dv["value"]:
                            # nothing was written since the process read it.  (A list
                            # with repeated keys can be a strict inflation of itself —
                            # keyfind pairs a later entry with the first one, whose ids
                            # differ — and the reference's reader then re-fires forever;
                            # this synchronous model re-runs once per write instead.)
                            continue
                        if lattice.threshold_met(dv["type"], dv["value"], th):
                            proc["seen"][i] = dv["value"]
                            try:
                                proc["body"](proc["seen"])
                            except Exception:
                                # Function(Scope) raised: the lasp_process dies and binds
                                # nothing (its supervisor's restarts re-read from scratch
                                # and crash the same way; lasp_process_sup.erl:57-60)
                                self.procs.remove(proc)
                            changed = True
        finally:
            self._depth -= 1

    def _bind_out(self, acc_id, acc_value):
        if acc_value is not None:
            self.bind(acc_id, acc_value)

    def union(self, l, r, out):
        t = self.vars[l]["type"]
        return self._start([l, r], lambda s: self._bind_out(out, union_body(t, s[l], s[r])))

    def intersection(self, l, r, out):
        t = self.vars[l]["type"]
        return self._start([l, r], lambda s: self._bind_out(out, intersection_body(t, s[l], s[r])))

    def product(self, l, r, out):
        t = self.vars[l]["type"]
        return self._start([l, r], lambda s: self._bind_out(out, product_body(t, s[l], s[r])))

    def map(self, i, fun, out):
        t = self.vars[i]["type"]
        return self._start([i], lambda s: self._bind_out(out, map_body(t, fun, s[i])))

    def filter(self, i, fun, out):
        t = self.vars[i]["type"]
        return self._start([i], lambda s: self._bind_out(out, filter_body(t, fun, s[i])))

    def fold(self, i, fun, out):
        t = self.vars[i]["type"]
        return self._start([i], lambda s: self._bind_out(out, fold_body(t, fun, s[i])))


def _normalise_threshold(t, threshold):
    """lasp_core.erl:339-346: undefined -> Type:new(); {strict, undefined} -> {strict, new()}."""
    if threshold is None:
        return type_mod(t).new()
    if isinstance(threshold, tuple) and len(threshold) == 2 and threshold[0] == "strict" \
            and threshold[1] is None:
        return ("strict", type_mod(t).new())
    return threshold


def _is_inflation(t, prev, cur):
    if t == "riak_dt_gcounter":
        return lattice.is_inflation(t, prev, cur)
    return lattice.is_inflation(t, prev, cur)


def _canon(v):
    # orddict / ordset values as nested lists of tuples for =:= matching
    if isinstance(v, list):
        return [_canon(x) for x in v]
    if isinstance(v, tuple):
        return tuple(_canon(x) for x in v)
    return v
