"""lasp_core over the device: declare / bind / update / read and the combinator
processes, with every variable's value resident in HBM.

Mirrors src/lasp_core.erl:
  declare/3 :208-218   bind/3 :291-312   update/4 :283-287   read/6 :331-364
  union/7 :602-627   intersection/7 :546-589   product/7 :499-533
  map/6 :641-667   filter/6 :681-712   fold/6 :460-486
  lasp_process:process/3 (src/lasp_process.erl:61-95) — the re-run-on-every-change loop,
  run synchronously: after each write, every process whose input is now a strict
  inflation of the value it last read re-runs its body on the device and binds the
  result.

All OR-Set variables of a Store share one element/token dictionary (codec.Domain), as
do all G-Set variables, so joins, predicates and combinators never re-map slots.
A variable holds one of two representations:
  canonical   an OR-Set / G-Set batch (16-byte {p, r} cells / bit words): the value is
              an orddict / ordset, and merge, equal and inflation are bit operations;
  list        a LIST batch (engine.ListBatch): the value exactly as a list — entries in
              list order, token runs in list order — for the non-canonical values the
              combinator bodies bind (intersection `Cx ++ Cy`, reversed product token
              pairs, reordered / repeated map and fold keys, the G-Set `L ++ R`).
A bind whose sides are both canonical uses the cell kernels; otherwise both sides are
lists (a canonical side converted on the device, laspj_list_from_set) and the bind is
the reference's own sequence — `Value0 =:= Value` (laspj_list_equal), Type:merge
(laspj_list_merge: orddict:merge / ordsets:union as written), is_inflation
(laspj_list_inflation) — so every re-run's output is merged exactly as lasp_core
merges it, duplicates and interleavings included.  Values are never updated in place
(every merge writes a new batch), so processes keep references to what they read.
"""

from __future__ import annotations

from typing import Callable, Dict, List, Optional

import numpy as np

from . import _lib, engine
from . import lists as L
from .codec import CapacityError, Domain, NonCanonical, _check_canonical_gset, \
    _check_canonical_orset
from .orset import context


class Unsupported(Exception):
    """A value or type this device store does not represent (documented in DESIGN.md)."""


class BodyCrash(Exception):
    """A combinator body raised (its fun failed on a key of the input): the reference's
    process crashes and binds nothing."""


class _Var:
    __slots__ = ("type", "rep", "val", "empty", "waiting", "pairs", "as_list", "gshape",
                 "last_write")

    def __init__(self, type_, val):
        self.type = type_
        self.rep = "canonical"
        self.val = val            # device batch (canonical) or engine.ListBatch (list)
        self.empty = True         # still new() = []
        self.waiting: List = []
        self.pairs = False        # list keys are product pairs {X, Y}
        self.as_list = None       # (value object, its list form) cache
        # lasp_orset_gbtree: {hkey(elem): token tree} of the elements whose token tree
        # is not ascending-insert shaped (gb_trees_ext:merge keeps a one-sided element's
        # tree as it is); the device holds the contents
        self.gshape: Dict = {}
        # (value before, value after) of the latest canonical merge that changed the value
        self.last_write = None


class _Value:
    """A device value about to be bound, or last read by a process."""
    __slots__ = ("rep", "batch", "pairs", "empty", "gb")

    def __init__(self, rep, batch, pairs=False, empty=None, gb=None):
        self.rep, self.batch, self.pairs, self.empty = rep, batch, pairs, empty
        self.gb = gb              # lasp_orset_gbtree: orset_gbtree.shape_info of the term


class Store:
    def __init__(self, capacity: int = 4096, ctx: Optional[engine.Context] = None,
                 token_words: int = 16):
        self.ctx = ctx or context()
        self.cap = capacity
        # an OR-Set element holds up to 64 * token_words tokens: a variable whose value
        # names a token slot >= 64 moves to wide cells (LASPJ_KIND_ORSET_WIDE, k {p, r}
        # pairs per element); the others keep 16-byte cells
        self.odom = Domain(element_capacity=capacity, token_capacity=64 * token_words)
        self.gdom = Domain(element_capacity=capacity)
        self.cdom = Domain(element_capacity=capacity)      # G-Counter actors
        self.ospace = L.ListSpace(self.ctx, self.odom, tokens=True)
        self.gspace = L.ListSpace(self.ctx, self.gdom, tokens=False)
        self.vars: Dict = {}
        self.procs: List[dict] = []
        self._n = 0
        self._depth = 0
        self._bottoms: Dict = {}
        # canonical batch -> its list form, for the bodies' operands: a stored batch is
        # never written again (updates and binds make new ones), so the conversion of a
        # value the bodies see again (the unchanged input of a re-run) is reused
        self._lcache: Dict = {}

    # ---------------------------------------------------------------- helpers
    def _new_batch(self, type_, k: int = 1):
        if type_ in ("lasp_orset", "lasp_orset_gbtree"):
            if k > 1:
                return self.ctx.orset_wide_batch(1, self.cap, k)
            return self.ctx.orset_batch(1, self.cap)
        if type_ == "lasp_gset":
            return self.ctx.gset_batch(1, self.cap)
        if type_ == "riak_dt_gcounter":
            return self.ctx.gcounter_batch(1, self.cap)
        raise Unsupported(type_)

    def _dom(self, type_) -> Domain:
        return self.gdom if type_ == "lasp_gset" else self.odom

    def _space(self, type_) -> L.ListSpace:
        return self.gspace if type_ == "lasp_gset" else self.ospace

    def _encode(self, type_, term, pairs: bool = False) -> _Value:
        """A host term as a device value: canonical when it is an orddict / ordset (and
        the variable holds no product pairs), else a list.

        A value the device form cannot hold — an element with more than 64 * token_words
        distinct tokens, or more distinct elements than the store's `capacity` — raises
        `Unsupported`, and the dictionary slots the attempt registered are undone.  The
        reference's merge takes such values (add_elem mints a fresh token per add,
        lasp_orset.erl:222-230, 261-262), so lasp_core:bind/3 would write them
        (lasp_core.erl:300-304): the store must not answer `ok` with the variable
        unchanged, which is what swallowing the error as a failed merge would do."""
        dom = self.cdom if type_ == "riak_dt_gcounter" else self._dom(type_)
        try:
            with dom.journal():
                return self._encode_term(type_, term, pairs)
        except CapacityError as e:
            raise Unsupported(f"value not representable on the device store: {e}") from e

    def _encode_term(self, type_, term, pairs: bool) -> _Value:
        if type_ == "riak_dt_gcounter":
            b = self._new_batch(type_)
            host = np.zeros((1, self.cap), dtype=np.uint64)
            for actor, n in term:
                host[0, self.cdom.element_slot(actor)] = n
            b.upload(host)
            return _Value("canonical", b, empty=not term)
        if type_ == "lasp_orset_gbtree":
            from .orset_gbtree import shape_info, to_orddict
            od = to_orddict(term)
            b = self._orset_upload(type_, od)
            return _Value("canonical", b, empty=not od, gb=shape_info(term))
        if not pairs:
            try:
                if type_ == "lasp_orset":
                    _check_canonical_orset(term)
                    ok = all(isinstance(f, bool) for _e, ts in term for _t, f in ts)
                else:
                    _check_canonical_gset(term)
                    ok = True
            except (NonCanonical, TypeError, ValueError):
                ok = False
            if ok:
                if type_ == "lasp_orset":
                    b = self._orset_upload(type_, term)
                else:
                    b = self._new_batch(type_)
                    b.upload(self.gdom.encode_gset([term], self.cap))
                return _Value("canonical", b, empty=not term)
        keys, toff, toks = L.encode(self._dom(type_), term, type_ == "lasp_gset", pairs)
        kind = _lib.KIND_GSET_LIST if type_ == "lasp_gset" else _lib.KIND_ORSET_LIST
        lb = engine.ListBatch(self.ctx, kind).upload(keys, toff, toks)
        return _Value("list", lb, pairs, empty=not term)

    def _orset_upload(self, type_, od):
        """An orddict in 16-byte cells, or in wide cells when it names a token slot >= 64."""
        k = self.odom.orset_words([od])
        b = self._new_batch(type_, k)
        if k == 1:
            b.upload(self.odom.encode_orset([od], self.cap))
        else:
            b.upload(self.odom.encode_orset_wide([od], self.cap, k))
        return b

    def _match(self, a, b):
        """Two OR-Set batches with one cell width (the narrower widened on the device,
        laspj_orset_widen: a new batch, the stored one untouched)."""
        k = max(_width(a), _width(b))
        return self._widen(a, k), self._widen(b, k)

    def _widen(self, b, k: int):
        if _width(b) >= k:
            return b
        return self.ctx.orset_wide_batch(b.replicas, b.elements, k).widen_from(b)

    def _decode_orset(self, b) -> list:
        cells = b.download()[0]
        return self.odom.decode_orset_wide(cells) if _width(b) > 1 else \
            self.odom.decode_orset(cells)

    def _to_list(self, type_, batch):
        """A canonical batch as a list (laspj_list_from_set)."""
        if _width(batch) > 1:
            raise Unsupported("a list form of an OR-Set value with more than 64 tokens "
                              "on an element")
        eb, n, tb = self._space(type_).set_orders(batch.elements)
        return engine.ListBatch.from_set(batch, eb, n, tb)

    def _var_list(self, v: _Var):
        if v.rep == "list":
            return v.val
        c = v.as_list
        if c is None or c[0] is not v.val:
            c = v.as_list = (v.val, self._to_list(v.type, v.val))
        return c[1]

    def _value_list(self, type_, dv: _Value):
        if dv.rep == "list":
            return dv.batch
        c = self._lcache.get(id(dv.batch))
        if c is not None and c[0] is dv.batch:
            return c[1]
        lst = self._to_list(type_, dv.batch)
        if len(self._lcache) >= 16:                     # oldest out (dicts keep order)
            self._lcache.pop(next(iter(self._lcache)))
        self._lcache[id(dv.batch)] = (dv.batch, lst)    # the entry keeps the batch alive
        return lst

    def _order(self, type_):
        return self._space(type_).order()

    def _is_empty(self, dv: _Value, type_) -> bool:
        if dv.empty is not None:
            return dv.empty
        if dv.rep == "list":
            return int(dv.batch.counts()[0][0]) == 0
        return bool(dv.batch.equal(self._bottom(type_, _width(dv.batch)))[0])

    def _bottom(self, type_, k: int = 1):
        b = self._bottoms.get((type_, k))
        if b is None:
            b = self._bottoms[(type_, k)] = self._new_batch(type_, k)
        return b

    # ---------------------------------------------------------------- declare / bind
    def declare(self, type_, id_=None):
        """declare/3 — lasp_core.erl:208-218 (idempotent)."""
        if id_ is None:
            self._n += 1
            id_ = f"var{self._n}".encode()
        if id_ not in self.vars:
            self.vars[id_] = _Var(type_, self._new_batch(type_))
        return ("ok", id_)

    def bind(self, id_, value):
        """bind/3 — lasp_core.erl:291-312.  `value` is a host term or a device value
        produced by a combinator body (`_Value`)."""
        v = self.vars[id_]
        try:
            dv = value if isinstance(value, _Value) else self._encode(v.type, value, v.pairs)
            self._bind_device(id_, v, dv)
        except (NonCanonical, ValueError, TypeError):
            # merge may throw for invalid values; bind swallows it (:308-311).  Values the
            # device cannot hold raise Unsupported from _encode instead (not swallowed).
            pass
        except _lib.LaspjError as e:
            if e.status in (_lib.E_UNSUPPORTED, _lib.E_NOMEM, _lib.E_DEVICE):
                raise Unsupported(str(e)) if e.status == _lib.E_UNSUPPORTED else e
        return ("ok", (id_, v.type, value))

    def bind_many(self, pairs):
        """Many binds as few device launches (laspj_batch_bind_many): every pair
        (id, term) whose variable and value are canonical is encoded, then ONE kernel
        does `Value0 =:= Value` + merge + write for all of them and ONE status download
        says which variables were written (lasp_core.erl:291-312 for each); other pairs
        bind one by one.  A variable named more than once takes its pairs in order, one
        per launch.  Every write lands first and the dataflow then runs once over all of
        them — one of the interleavings the reference's asynchronous processes allow
        (its lasp_process readers race with binds).  Schedules are observable (the union
        body keeps the left side's tokens, and re-runs merge into the output), so this is
        that interleaving: the binds in pair order with propagation deferred to the end,
        not the one-bind-at-a-time one."""
        allp = list(pairs)                        # (a generator is read once)
        self._depth += 1                          # one propagation after all writes
        done = False
        try:
            todo = allp
            while todo:
                pend, seen, later = [], set(), []
                for id_, term in todo:
                    if id_ in seen:               # this variable's next pair: next launch
                        later.append((id_, term))
                        continue
                    seen.add(id_)
                    v = self.vars[id_]
                    if v.type in ("lasp_orset", "lasp_gset", "riak_dt_gcounter") and \
                            v.rep == "canonical" and not v.empty:
                        try:
                            dv = self._encode(v.type, term, v.pairs)
                        except (NonCanonical, ValueError, TypeError):
                            continue              # merge would throw: bind swallows it
                        if dv.rep == "canonical":
                            pend.append((id_, v, dv))
                            continue
                    self.bind(id_, term)          # written now, propagated at the end
                if pend:
                    ops = [self._match(v.val, d.batch) for _i, v, d in pend]
                    dsts = [_new_like(self.ctx, c) for c, _n in ops]
                    st = self.ctx.bind_many(dsts, [c for c, _n in ops], [n for _c, n in ops])
                    for (id_, v, _d), dst, s_ in zip(pend, dsts, st):
                        if s_:
                            v.val = dst
                            self._written(id_, v)
                todo = later
            done = True
        finally:
            self._depth -= 1
            # the writes that landed before a failure still reach their processes
            if done:
                self._propagate()
            else:
                try:
                    self._propagate()
                except Exception:                 # the original error is the one raised
                    pass
        return [("ok", (i, self.vars[i].type, t)) for i, t in allp]

    def _bind_device(self, id_, v: _Var, dv: _Value):
        t = v.type
        if v.empty:
            # Value0 = new() = []: `[] =:= Value` is a no-op; otherwise merge([], V) = V
            # (orddict:merge([], D) = D, ordsets:union([], S) = S) and it inflates []
            if self._is_empty(dv, t):
                return
            v.rep, v.val, v.pairs = dv.rep, dv.batch, dv.pairs
            v.empty = False
            if t == "lasp_orset_gbtree" and dv.gb is not None:
                v.gshape = dict(dv.gb[1])            # merge(empty(), V) keeps V's trees
            self._written(id_, v)
            return
        if v.rep == "canonical" and dv.rep == "canonical":
            cur, new = self._match(v.val, dv.batch)
            if t != "lasp_orset_gbtree":
                # `Value0 =:= Value` + merge in one launch (laspj_batch_bind_many); a
                # canonical merge always inflates Value0, so it is written (:301-303)
                merged = _new_like(self.ctx, cur)
                if not self.ctx.bind_many([merged], [cur], [new])[0]:
                    return                                       # lasp_core.erl:294-296
                # merged came from v.val by a merge that changed it: a strict inflation
                # of v.val, which _propagate then knows without asking the device
                v.last_write = (v.val, merged)
                v.val = merged
                self._written(id_, v)
                return
            same = bool(cur.equal(new)[0])
            if t == "lasp_orset_gbtree" and dv.gb is not None:
                # `case Value0 of Value` matches whole terms: the stored value's outer
                # tree is ascending-insert shaped (a merge output), so Value must be too,
                # with the same token-tree shapes
                outer, odd, _keys = dv.gb
                same = same and outer and _same_shapes(v.gshape, odd)
            if same:                                             # lasp_core.erl:294-296
                return
            merged = _new_like(self.ctx, cur)
            _or_into(self.ctx, merged, cur, new)
            if not bool(merged.is_inflation_of(cur)[0]):         # lasp_core.erl:301
                return
            if t == "lasp_orset_gbtree" and dv.gb is not None:
                # gb_trees_ext:merge/3: an element of both operands gets an ascending
                # token tree, one of one operand keeps that operand's tree
                from .terms import hkey
                old_keys = {hkey(e) for e, _ts in self._decode_orset(cur)}
                _outer, odd, new_keys = dv.gb
                v.gshape = {k: tr for k, tr in v.gshape.items() if k not in new_keys}
                v.gshape.update({k: tr for k, tr in odd.items() if k not in old_keys})
            v.val = merged
            self._written(id_, v)
            return
        if t not in ("lasp_orset", "lasp_gset"):
            raise Unsupported(f"list values of {t}")
        if dv.pairs != v.pairs and not self._is_empty(dv, t):
            # product pairs meet plain keys: the rank tables do not order the two
            raise Unsupported("a product output and plain keys in one variable")
        old, new = self._var_list(v), self._value_list(t, dv)
        order = self._order(t)
        # Value0 =:= Value -> no-op; Merged = Type:merge(Value0, Value); write when
        # is_inflation(Value0, Merged) — one call (laspj_list_bind)
        merged, st = old.bind(new, order)
        if st[0] != 1:
            return
        v.rep, v.val = "list", merged
        self._written(id_, v)

    def _written(self, id_, v: _Var):
        # write/4 + reply_to_all/3 (lasp_core.erl:839-844, 765-825)
        v.waiting = [th for th in v.waiting if not self._threshold_met(v, th)]
        self._propagate()

    # ---------------------------------------------------------------- update / read
    def update(self, id_, op, actor):
        """update/4 — lasp_core.erl:283-287: Type:update on the value, then bind."""
        v = self.vars[id_]
        if v.rep != "canonical":
            raise Unsupported("update/3 on a combinator output (a list value)")
        from . import orset as _o
        ops, script = [], []
        dom = self.cdom if v.type == "riak_dt_gcounter" else self._dom(v.type)
        try:
            # the op's slots (the 65th token of an element — add_elem mints one per add,
            # lasp_orset.erl:222-230 — or an element past `capacity` is Unsupported, and
            # the slots the op registered are undone)
            with dom.journal():
                if v.type == "riak_dt_gcounter":
                    from .gcounter import increment_amount
                    ops.append((0, self.cdom.element_slot(actor), increment_amount(op)))
                elif v.type == "lasp_orset":
                    _o._compile(op, self.odom, ops, new_call=True)
                elif v.type == "lasp_orset_gbtree":
                    from . import orset_gbtree as _og
                    _og._compile(op, self.odom, ops, new_call=True, script=script)
                else:
                    elems = [op[1]] if op[0] == "add" else list(op[1])
                    ops = [(0, self.gdom.element_slot(e), _lib.OP_ADD, 0, 1) for e in elems]
        except CapacityError as e:
            raise Unsupported(f"update not representable on the device store: {e}") from e
        k = 1
        if v.type in ("lasp_orset", "lasp_orset_gbtree"):
            k = max([_width(v.val)] + [(o[3] >> 6) + 1 for o in ops if o[2] != _lib.OP_REMOVE])
        if k > _width(v.val):
            cur = self._widen(v.val, k)       # the op mints token slot >= 64 * width
        else:
            cur = _new_like(self.ctx, v.val)
            _or_into(self.ctx, cur, v.val, v.val)
        if v.type == "riak_dt_gcounter":
            cur.increment(ops)
        elif v.type == "lasp_orset" and all(o[2] == _lib.OP_ADD for o in ops):
            # add / add_by_token / add_all: no precondition can fail (lasp_orset.erl:
            # 222-230), so no statuses are read back and nothing waits for the device
            cur.apply_ops(ops, statuses=False)
        elif v.type in ("lasp_orset", "lasp_orset_gbtree"):
            st = cur.apply_ops(ops)
            if (st == _lib.OPST_KEY_EXISTS).any():
                j = int(np.nonzero(st == _lib.OPST_KEY_EXISTS)[0][0])
                from .orset_gbtree import KeyExists
                raise KeyExists(self.odom.tokens[ops[j][1]].terms[ops[j][3]])
            if (st == _lib.OPST_NOT_PRESENT).any():
                bad = ops[int(np.nonzero(st == _lib.OPST_NOT_PRESENT)[0][0])][1]
                raise RuntimeError(f"badmatch: {{error,{{precondition,{{not_present,"
                                   f"{self.odom.elements.terms[bad]!r}}}}}}}")
        else:
            cur.apply_ops(ops, statuses=False)             # G-Set adds: nothing can fail
        gb = None
        if v.type == "lasp_orset_gbtree":
            # Type:update's tree (its insert / enter calls replayed on the stored tree),
            # then bind/3 merges it into the stored value
            from .orset_gbtree import _replay, shape_info
            gb = shape_info(_replay(script, self.value(id_)))
        self._bind_device(id_, v, _Value("canonical", cur, empty=False, gb=gb))
        return ("ok", (id_, v.type, None))

    def read(self, id_, threshold=("strict", None)):
        """read/6 — lasp_core.erl:331-364 (non-blocking: None and a recorded waiter)."""
        v = self.vars[id_]
        bottom = _type_new(v.type)
        if threshold is None:
            threshold = bottom                            # Type:new()
        elif isinstance(threshold, tuple) and threshold[0] == "strict" and threshold[1] is None:
            threshold = ("strict", bottom)
        if self._threshold_met(v, threshold):
            return ("ok", (id_, v.type, self.value(id_)))
        if threshold not in v.waiting:       # one pending entry per distinct threshold
            v.waiting.append(threshold)
        return None

    def _threshold_met(self, v: _Var, threshold) -> bool:
        """lasp_lattice:threshold_met/3 on the device (lasp_lattice.erl:62-75)."""
        strict = isinstance(threshold, tuple) and len(threshold) == 2 and \
            threshold[0] == "strict"
        term = threshold[1] if strict else threshold
        if v.type == "riak_dt_gcounter":
            # Threshold =< value(V) (lasp_lattice.erl:87-90): term-order cases on the
            # host (gcounter.threshold_plan), the sum compared on the device
            from .gcounter import threshold_plan
            const, t = threshold_plan(term, strict)
            if const is not None:
                return const
            return bool(v.val.threshold_met(t, False)[0])
        return self._inflates(v, self._encode(v.type, term, v.pairs), strict)

    def _inflates(self, v: _Var, prev: _Value, strict: bool) -> bool:
        """is_inflation(prev, V) / is_strict_inflation(prev, V) for V = v's value."""
        if v.rep == "canonical" and prev.rep == "canonical":
            cur, pb = self._match(v.val, prev.batch)
            if bool(cur.is_inflation_of(pb, strict=strict)[0]):
                return True
            if strict and v.type == "lasp_orset_gbtree" and prev.gb is not None:
                # `Ids =/= Ids1` (lasp_lattice.erl:217-233) compares token TREES: a
                # common element whose tree has another shape is changed too
                from .gbtrees import shape
                from .terms import hkey
                _outer, odd, keys = prev.gb
                common = keys & {hkey(e) for e, _t in self._decode_orset(v.val)}
                differs = any((k in odd) != (k in v.gshape) or
                              (k in odd and shape(odd[k]) != shape(v.gshape[k]))
                              for k in common)
                return differs and bool(cur.is_inflation_of(pb)[0])
            return False
        if v.type not in ("lasp_orset", "lasp_gset"):
            raise Unsupported(f"list values of {v.type}")
        cur = self._var_list(v)
        return bool(cur.is_inflation_of(self._value_list(v.type, prev), self._order(v.type),
                                        strict=strict)[0])

    def value(self, id_):
        """The variable's value as the reference would hold it (decoded from HBM)."""
        v = self.vars[id_]
        if v.rep == "list":
            keys, toff, toks = v.val.download()
            return L.decode(self._dom(v.type), keys, toff, toks, v.type == "lasp_gset")
        if v.type == "lasp_orset_gbtree":
            from .orset_gbtree import with_shapes
            return with_shapes(self._decode_orset(v.val), v.gshape)
        if v.type == "lasp_orset":
            return self._decode_orset(v.val)
        cells = v.val.download()[0]
        if v.type == "riak_dt_gcounter":
            return [(self.cdom.elements.terms[int(a)], int(cells[int(a)]))
                    for a in self.cdom.elements.order() if int(cells[int(a)])]
        return self.gdom.decode_gset(cells)

    def type_value(self, id_):
        """Type:value(Value) of the variable (value/1 kernel + decode)."""
        v = self.vars[id_]
        if v.type == "riak_dt_gcounter":
            return int(v.val.values()[0])
        if v.type == "lasp_gset":
            return self.value(id_)
        if v.rep == "list":
            keys, _o, _t = v.val.value().download()
            return [L._key_term(self.odom, int(k)) for k in keys]
        return self.odom.decode_value_bits(v.val.value_bits()[0])

    # ---------------------------------------------------------------- processes
    def _start(self, inputs, body):
        for i in inputs:
            if self.vars[i].type not in ("lasp_orset", "lasp_gset"):
                # lasp_core's combinator bodies match the orddict shape and the
                # lasp_orset / lasp_gset atoms only (lasp_core.erl:460-712)
                raise Unsupported("combinators take lasp_orset / lasp_gset inputs")
        proc = {"inputs": list(inputs), "seen": {i: None for i in inputs}, "body": body}
        self.procs.append(proc)
        self._propagate()
        return "ok"

    def _propagate(self):
        self._depth += 1
        if self._depth > 1:
            self._depth -= 1
            return
        try:
            changed = True
            while changed:
                changed = False
                pre = self._strict_checks()
                for proc in list(self.procs):
                    for i in proc["inputs"]:
                        if proc not in self.procs:
                            break
                        v = self.vars[i]
                        last = proc["seen"][i]
                        if v.empty:
                            continue
                        # {strict, new()}: a non-empty value is a strict inflation of []
                        if last is not None:
                            if last.batch is v.val:
                                # unchanged since read: one re-run per write (a list
                                # with repeated keys can strictly inflate itself, on
                                # which the reference's reader re-fires forever;
                                # DESIGN.md §2)
                                continue
                            hit = pre.get((id(proc), i))
                            if self._merged_from(v, last):
                                fire = True
                            elif hit is not None and hit[0] is v.val and hit[2] is last.batch:
                                fire = hit[1]
                            else:
                                fire = self._inflates(v, last, strict=True)
                            if not fire:
                                continue
                        proc["seen"][i] = _Value(v.rep, v.val, v.pairs, empty=False)
                        try:
                            proc["body"](proc["seen"])
                        except BodyCrash:
                            # the process dies: nothing bound, no more re-runs
                            self.procs.remove(proc)
                        changed = True
        finally:
            self._depth -= 1

    @staticmethod
    def _merged_from(v: _Var, last) -> bool:
        """v's value is a canonical merge that changed last's value: for lasp_orset,
        lasp_gset and riak_dt_gcounter a strict inflation of it (changed cells of a merge
        = a new element, a token or flag gained on a common element, a larger count:
        lasp_lattice.erl:212-215, 235-253, 273-275), known without a device call."""
        lw = getattr(v, "last_write", None)
        return lw is not None and lw[1] is v.val and lw[0] is last.batch and \
            v.type in ("lasp_orset", "lasp_gset", "riak_dt_gcounter") and \
            v.rep == "canonical" and last.rep == "canonical"

    def _strict_checks(self):
        """Every pending {strict, Last} re-check between canonical values, in ONE
        launch (laspj_batch_inflation_many): {(proc, input): (value, result, last)}."""
        keys, prevs, curs = [], [], []
        for proc in self.procs:
            for i in proc["inputs"]:
                v, last = self.vars[i], proc["seen"][i]
                if v.empty or last is None or last.batch is v.val or self._merged_from(v, last):
                    continue
                if v.rep == "canonical" and last.rep == "canonical" and \
                        v.type in ("lasp_orset", "lasp_gset", "riak_dt_gcounter") and \
                        _width(v.val) == _width(last.batch):
                    keys.append(((id(proc), i), v.val, last.batch))
                    prevs.append(last.batch)
                    curs.append(v.val)
        if len(keys) < 2:
            return {}
        res = self.ctx.inflation_many(prevs, curs, strict=True)
        return {k: (val, bool(r), lb) for (k, val, lb), r in zip(keys, res)}

    def _bind_out(self, out_id, dv):
        if dv is not None:
            self.bind(out_id, dv)

    def _lists(self, t, *vals):
        return [self._value_list(t, x) for x in vals]

    @staticmethod
    def _run(fn, *args):
        try:
            return fn(*args)
        except _lib.LaspjError as e:
            if e.status == _lib.E_FUN:
                raise BodyCrash(str(e)) from e
            raise

    def union(self, l, r, out):
        t = self.vars[l].type

        def body(seen):
            a, b = seen[l], seen[r]
            if a is None or b is None:
                return
            if t == "lasp_orset" and a.rep == b.rep == "canonical":
                _narrow(a.batch, b.batch)
                res = self._new_batch(t).union(a.batch, b.batch)       # keep-left merge
                return self._bind_out(out, _Value("canonical", res))
            _pairs_guard(a, b)
            la, lb = self._lists(t, a, b)
            # OR-Set: orddict:merge keep-left; G-Set: LValue ++ RValue
            self._bind_out(out, _Value("list", la.union(lb, self._order(t)), a.pairs))
        return self._start([l, r], body)

    def intersection(self, l, r, out):
        t = self.vars[l].type

        def body(seen):
            a, b = seen[l], seen[r]
            if a is None or b is None:
                return
            self._gset_tuples_guard(t, a, b)
            if t == "lasp_gset" and a.rep == b.rep == "canonical":
                res = self._new_batch(t).intersection(a.batch, b.batch)
                return self._bind_out(out, _Value("canonical", res))
            _pairs_guard(a, b)
            if b.rep == "canonical" and _width(b.batch) == 1:
                # keyfind in R's list form = R's cell of the key's slot: R is read in place
                # (laspj_list_intersection_set), not converted
                la = self._value_list(t, a)
                _eb, _n, tb = self._space(t).set_orders(b.batch.elements)
                self._order(t)                    # (rank tables current for the bind)
                return self._bind_out(out, _Value("list", la.intersection_set(b.batch, tb),
                                                  a.pairs))
            la, lb = self._lists(t, a, b)
            self._bind_out(out, _Value("list", la.intersection(lb, self._order(t)), a.pairs))
        return self._start([l, r], body)

    def product(self, l, r, out):
        t = self.vars[l].type

        def body(seen):
            a, b = seen[l], seen[r]
            if a is None or b is None:
                return
            self._gset_tuples_guard(t, a, b)
            la, lb = self._lists(t, a, b)
            self._bind_out(out, _Value("list", la.product(lb), True))
        return self._start([l, r], body)

    def filter(self, i, fun: Callable, out):
        t = self.vars[i].type
        fc = L.FunCache(fun)
        dom = self._dom(t)

        def body(seen):
            a = seen[i]
            if a.rep == "canonical":
                keep = L.filter_table(fc, dom.elements.terms, t == "lasp_gset")
                if not (keep == 2).any():
                    bits = np.zeros(((self.cap + 63) // 64,), dtype=np.uint64)
                    for e in np.nonzero(keep == 1)[0]:
                        bits[e >> 6] |= np.uint64(1) << np.uint64(e & 63)
                    _narrow(a.batch)
                    res = self._new_batch(t).filter(a.batch, bits)
                    return self._bind_out(out, _Value("canonical", res))
            la = self._value_list(t, a)
            terms, per_entry = L.table_terms(dom, la, a.pairs)
            keep = L.filter_table(fc, terms, t == "lasp_gset")
            self._bind_out(out, _Value("list", self._run(la.filter, keep, per_entry), a.pairs))
        return self._start([i], body)

    def map(self, i, fun: Callable, out):
        t = self.vars[i].type
        fc = L.FunCache(fun)
        dom = self._dom(t)

        def body(seen):
            la = self._value_list(t, seen[i])
            terms, per_entry = L.table_terms(dom, la, seen[i].pairs)
            keys = L.map_table(dom, fc, terms, t == "lasp_gset")
            self._bind_out(out, _Value("list", self._run(la.map, keys, per_entry)))
        return self._start([i], body)

    def fold(self, i, fun: Callable, out):
        t = self.vars[i].type
        fc = L.FunCache(fun)
        dom = self._dom(t)

        def body(seen):
            la = self._value_list(t, seen[i])
            terms, per_entry = L.table_terms(dom, la, seen[i].pairs)
            off, keys = L.fold_table(dom, fc, terms, t == "lasp_gset")
            self._bind_out(out, _Value("list", self._run(la.fold, off, keys, per_entry)))
        return self._start([i], body)

    def _gset_tuples_guard(self, t, a: _Value, b: _Value):
        """lasp_core's intersection / product bodies match `{X, Causality}` first
        (lasp_core.erl:513-521, 560-576): a G-Set holding 2-tuples goes down the OR-Set
        branch (keyfind and `++` on the tuples' second elements), which this store does
        not reproduce."""
        if t != "lasp_gset":
            return
        if a.pairs or b.pairs or any(isinstance(x, tuple) and len(x) == 2
                                     for x in self.gdom.elements.terms):
            raise Unsupported("G-Set intersection / product over 2-tuple elements")


def _pairs_guard(a: _Value, b: _Value):
    if a.pairs != b.pairs:
        raise Unsupported("a product output and plain keys in one combinator")


def _same_shapes(a: Dict, b: Dict) -> bool:
    """Two {hkey: token tree} maps name the same elements with trees of one shape."""
    from .gbtrees import shape
    return a.keys() == b.keys() and all(shape(a[k]) == shape(b[k]) for k in a)


def _type_new(type_):
    """Type:new() (lasp_core.erl:339-346 substitutes it for an undefined threshold)."""
    if type_ == "lasp_orset_gbtree":
        from .gbtrees import empty
        return empty()
    return []


def _width(b) -> int:
    """{p, r} pairs per cell of an OR-Set batch (1 for narrow cells and other kinds)."""
    return getattr(b, "token_words", 1)


def _narrow(*bs):
    if any(_width(b) > 1 for b in bs):
        raise Unsupported("combinator bodies over an OR-Set value with more than 64 tokens "
                          "on an element")


def _new_like(ctx, b):
    """An empty batch of b's kind and shape."""
    if isinstance(b, engine.ORSetWideBatch):
        return ctx.orset_wide_batch(b.replicas, b.elements, b.token_words)
    out = type(b).__new__(type(b))
    engine._Batch.__init__(out, ctx, b.replicas, b.elements)
    return out


def _or_into(ctx, dst, a, b):
    """dst := a ⊔ b slot-wise: one k_or16 launch, or the per-actor max for G-Counters."""
    if isinstance(dst, engine.GCounterBatch):
        _lib.check(ctx.L.laspj_gcounter_join(ctx.h, dst.h, a.h, b.h), ctx.h)
    else:
        _lib.check(ctx.L.laspj_batch_join(ctx.h, dst.h, a.h, b.h), ctx.h)
