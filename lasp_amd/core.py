"""lasp_core over the device: declare / bind / update / read and the combinator
processes, with every variable's value resident in HBM.

Mirrors src/lasp_core.erl:
  declare/3 :208-218   bind/3 :291-312   update/4 :283-287   read/6 :331-364
  union/7 :602-627   intersection/7 :546-589   product/7 :499-533
  map/6 :641-667   filter/6 :681-712   fold/6 :460-486
  lasp_process:process/3 (src/lasp_process.erl:61-95) — the re-run-on-every-change loop,
  run synchronously: after each write, every process whose input is now a strict
  inflation of the value it last read (a device inflation kernel) re-runs its body on
  the device and binds the result.

All OR-Set variables of a Store share one element/token dictionary (codec.Domain), as
do all G-Set variables, so joins, predicates and combinators never re-map slots.
A variable holds one of
  canonical   ORSetBatch / GSetBatch over the store dictionary,
  concat      the intersection body's {X, Cx ++ Cy} list (ConcatBatch),
  product     the product body's list (ORSetProductBatch / GSetProductBatch),
  seq         the map / fold body's list (a batch over SeqOutput slots, list order).
bind(Var, V): if Var still holds new(), the reference's merge(new(), V) is V itself
(orddict:merge([], D) = D, ordsets:union([], S) = S), so V is stored as is; otherwise
Var and V must have the same representation and are joined slot-wise on the device.
For canonical values that is exactly lasp_orset:merge/2; for seq values with
non-decreasing keys (map X -> 2X, fold X -> [X,X,X]) it equals orddict:merge's
positional pairing; for concat / product values the reference's two-finger merge of
unsorted token lists is not reproduced (parity unpinned there).
"""

from __future__ import annotations

from typing import Callable, Dict, List, Optional

import numpy as np

from . import _lib, engine
from .codec import Domain, NonCanonical, SeqOutput, decode_concat, decode_gset_product, \
    decode_product
from .orset import context
from .terms import hkey


class Unsupported(Exception):
    """A type that is not on the device path (the store holds lasp_orset / lasp_gset)."""


class _Var:
    __slots__ = ("type", "rep", "val", "seq", "empty", "waiting")

    def __init__(self, type_, val):
        self.type = type_
        self.rep = "canonical"
        self.val = val            # device batch
        self.seq: Optional[SeqOutput] = None
        self.empty = True         # still new()
        self.waiting: List = []


class Store:
    def __init__(self, capacity: int = 4096, ctx: Optional[engine.Context] = None):
        self.ctx = ctx or context()
        self.cap = capacity
        self.odom = Domain(element_capacity=capacity)
        self.gdom = Domain(element_capacity=capacity)
        self.cdom = Domain(element_capacity=capacity)      # G-Counter actors
        self.vars: Dict = {}
        self.procs: List[dict] = []
        self._n = 0
        self._depth = 0
        self._bottoms: Dict = {}

    # ---------------------------------------------------------------- helpers
    def _new_batch(self, type_):
        if type_ in ("lasp_orset", "lasp_orset_gbtree"):
            return self.ctx.orset_batch(1, self.cap)
        if type_ == "lasp_gset":
            return self.ctx.gset_batch(1, self.cap)
        if type_ == "riak_dt_gcounter":
            return self.ctx.gcounter_batch(1, self.cap)
        raise Unsupported(type_)

    def _encode(self, type_, term):
        b = self._new_batch(type_)
        if type_ == "lasp_orset_gbtree":
            from .orset_gbtree import to_orddict
            b.upload(self.odom.encode_orset([to_orddict(term)], self.cap))
        elif type_ == "lasp_orset":
            b.upload(self.odom.encode_orset([term], self.cap))
        elif type_ == "lasp_gset":
            b.upload(self.gdom.encode_gset([term], self.cap))
        else:
            host = np.zeros((1, self.cap), dtype=np.uint64)
            for actor, n in term:
                host[0, self.cdom.element_slot(actor)] = n
            b.upload(host)
        return b

    def _copy(self, b):
        """Device copy of a batch (x ⊔ x = x for canonical kinds, OR otherwise)."""
        out = type(b).__new__(type(b))
        if isinstance(b, engine._ProductBatch):
            engine._ProductBatch.__init__(out, self.ctx, b.replicas, b.elements, b.elements_r)
            out.kind = b.kind
        else:
            engine._Batch.__init__(out, self.ctx, b.replicas, b.elements)
        _or_into(self.ctx, out, b, b)
        return out

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
        produced by a combinator body (`_DeviceValue`)."""
        v = self.vars[id_]
        try:
            dv = value if isinstance(value, _DeviceValue) else \
                _DeviceValue("canonical", self._encode(v.type, value))
            self._bind_device(id_, v, dv)
        except (NonCanonical, _lib.LaspjError, ValueError):
            pass        # merge may throw for invalid values; bind swallows it (:308-311)
        return ("ok", (id_, v.type, value))

    def _is_bottom(self, v: _Var, dv: "_DeviceValue") -> bool:
        if dv.rep != "canonical":
            return False
        return bool(dv.batch.equal(self._bottom(v.type))[0])

    def _bottom(self, type_):
        b = self._bottoms.get(type_)
        if b is None:
            b = self._bottoms[type_] = self._new_batch(type_)
        return b

    def _bind_device(self, id_, v: _Var, dv: "_DeviceValue"):
        if v.empty:
            if self._is_bottom(v, dv):       # Value0 =:= Value = new(): no-op
                return
            # merge(new(), V) = V; is_inflation(new(), V) holds
            v.rep, v.seq, v.val = dv.rep, dv.seq, self._copy(dv.batch)
            v.empty = False
            self._written(id_, v)
            return
        if v.rep != dv.rep:
            raise ValueError("representation mismatch (merge would throw)")
        new = dv.batch
        if v.rep == "seq" and v.seq.keys != dv.seq.keys:
            new = self._align_seq(v, dv)
        # Value0 =:= Value: no-op (lasp_core.erl:294-296)
        if v.rep == "canonical" and bool(v.val.equal(new)[0]):
            return
        merged = self._copy(v.val)
        _or_into(self.ctx, merged, merged, new)
        if v.rep == "canonical":
            if not bool(merged.is_inflation_of(v.val)[0]):     # lasp_core.erl:301
                return
        v.val = merged
        self._written(id_, v)

    def _align_seq(self, v: _Var, dv: "_DeviceValue"):
        """Re-run outputs grow with the input dictionary: lay the new list out on the
        variable's slots extended by the new slots (keys and causality source match)."""
        old_keys = [(hkey(k) if s != 0xFFFFFFFF else None, s) for k, s in zip(v.seq.keys, v.seq.src)]
        new_keys = [(hkey(k) if s != 0xFFFFFFFF else None, s) for k, s in zip(dv.seq.keys, dv.seq.src)]
        # the k-th occurrence of (key, source slot) in the old layout moves to the k-th
        # occurrence in the new one; slots only the new layout has start empty
        pos = {}
        for o, k in enumerate(new_keys):
            pos.setdefault(k, []).append(o)
        idx = np.full((len(new_keys),), 0xFFFFFFFF, np.uint32)
        seen = {}
        for o, k in enumerate(old_keys):
            j = seen.get(k, 0)
            if j >= len(pos.get(k, [])):
                raise ValueError("map/fold layout changed incompatibly")
            idx[pos[k][j]] = o
            seen[k] = j + 1
        widened = self._batch_like(v.type, len(new_keys))
        widened.gather(v.val, idx)
        v.val, v.seq = widened, dv.seq
        return dv.batch

    def _batch_like(self, type_, n):
        return self.ctx.orset_batch(1, max(1, n)) if type_ == "lasp_orset" else \
            self.ctx.gset_batch(1, max(1, n))

    def _written(self, id_, v: _Var):
        # write/4 + reply_to_all/3 (lasp_core.erl:839-844, 765-825)
        still = []
        for th in v.waiting:
            if not self._threshold_met(v, th):
                still.append(th)
        v.waiting = still
        self._propagate()

    # ---------------------------------------------------------------- update / read
    def update(self, id_, op, actor):
        """update/4 — lasp_core.erl:283-287: Type:update on a copy, then bind."""
        v = self.vars[id_]
        if v.rep != "canonical":
            raise ValueError("badmatch: update on a combinator output")
        from . import orset as _o
        cur = self._copy(v.val)
        if v.type == "riak_dt_gcounter":
            from .gcounter import increment_amount
            n = increment_amount(op)
            cur.increment([(0, self.cdom.element_slot(actor), n)])
        elif v.type in ("lasp_orset", "lasp_orset_gbtree"):
            ops = []
            if v.type == "lasp_orset":
                _o._compile(op, self.odom, ops, new_call=True)
            else:
                from . import orset_gbtree as _og
                _og._compile(op, self.odom, ops, new_call=True)
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
            elems = [op[1]] if op[0] == "add" else list(op[1])
            cur.apply_ops([(0, self.gdom.element_slot(e), _lib.OP_ADD, 0, 1) for e in elems])
        self._bind_device(id_, v, _DeviceValue("canonical", cur))
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
        strict = isinstance(threshold, tuple) and threshold[0] == "strict"
        term = threshold[1] if strict else threshold
        if v.type == "riak_dt_gcounter":
            # Threshold =< value(V) (lasp_lattice.erl:87-90): term-order cases on the
            # host (gcounter.threshold_plan), the sum compared on the device
            from .gcounter import threshold_plan
            const, t = threshold_plan(term, strict)
            if const is not None:
                return const
            return bool(v.val.threshold_met(t, False)[0])
        if v.rep != "canonical":
            # combinator outputs are only read with the bottom threshold
            if term not in ([],):
                raise ValueError("threshold reads on combinator outputs take new()")
            return (not strict) or not v.empty
        t = self._encode(v.type, term)
        return bool(v.val.is_inflation_of(t, strict=strict)[0])

    def value(self, id_):
        """The variable's value as the reference would hold it (decoded from HBM)."""
        v = self.vars[id_]
        cells = v.val.download()[0]
        if v.type == "riak_dt_gcounter":
            return [(self.cdom.elements.terms[int(a)], int(cells[int(a)]))
                    for a in self.cdom.elements.order() if int(cells[int(a)])]
        if v.rep == "canonical":
            if v.type == "lasp_orset_gbtree":
                from .orset_gbtree import from_orddict
                return from_orddict(self.odom.decode_orset(cells))
            return self.odom.decode_orset(cells) if v.type == "lasp_orset" else \
                self.gdom.decode_gset(cells)
        if v.rep == "concat":
            return decode_concat(self.odom, cells)
        if v.rep == "product":
            return decode_product(self.odom, self.odom, cells) if v.type == "lasp_orset" \
                else decode_gset_product(self.gdom, self.gdom, cells)
        return v.seq.decode_orset(cells) if v.type == "lasp_orset" else v.seq.decode_bits(cells)

    def type_value(self, id_):
        """Type:value(Value) of the variable (value/1 kernel + decode)."""
        v = self.vars[id_]
        if v.type == "riak_dt_gcounter":
            return int(v.val.values()[0])
        if v.type == "lasp_gset":
            return self.value(id_)
        bits = v.val.value_bits()[0]
        if v.rep == "canonical":
            return self.odom.decode_value_bits(bits)
        if v.rep == "concat":
            return _concat_visible(self.odom, bits)
        if v.rep == "product":
            ER = v.val.elements_r
            return [(self.odom.elements.terms[x], self.odom.elements.terms[y])
                    for x in self.odom.elements.order() for y in self.odom.elements.order()
                    if (int(bits[(int(x) * ER + int(y)) >> 6]) >> ((int(x) * ER + int(y)) & 63)) & 1]
        return v.seq.decode_bits(bits)

    # ---------------------------------------------------------------- processes
    def _start(self, inputs, body):
        for i in inputs:
            if self.vars[i].type == "lasp_orset_gbtree":
                # lasp_core's combinator bodies match the orddict shape and the
                # lasp_orset / lasp_gset atoms only (lasp_core.erl:460-712): a gbtree
                # input crashes the process in the reference
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
                for proc in self.procs:
                    for i in proc["inputs"]:
                        v = self.vars[i]
                        last = proc["seen"][i]
                        if v.empty:
                            continue
                        if last is None:
                            # {strict, new()}: a non-empty value is a strict inflation
                            fire = True
                        elif v.rep == "canonical":
                            fire = bool(v.val.is_inflation_of(last, strict=True)[0])
                        else:
                            fire = False
                        if fire:
                            proc["seen"][i] = self._copy(v.val)
                            proc["body"](proc["seen"])
                            changed = True
        finally:
            self._depth -= 1

    def _bind_out(self, out_id, dv):
        if dv is not None:
            self.bind(out_id, dv)

    def union(self, l, r, out):
        t = self.vars[l].type

        def body(seen):
            if seen[l] is None or seen[r] is None:
                return
            res = self._new_batch(t)
            if t == "lasp_orset":
                res.union(seen[l], seen[r])
            else:
                res.union(seen[l], seen[r])
            self._bind_out(out, _DeviceValue("canonical", res))
        return self._start([l, r], body)

    def intersection(self, l, r, out):
        t = self.vars[l].type

        def body(seen):
            if seen[l] is None or seen[r] is None:
                return
            if t == "lasp_orset":
                self._bind_out(out, _DeviceValue("concat", seen[l].intersection(seen[r])))
            else:
                res = self._new_batch(t).intersection(seen[l], seen[r])
                self._bind_out(out, _DeviceValue("canonical", res))
        return self._start([l, r], body)

    def product(self, l, r, out):
        def body(seen):
            if seen[l] is None or seen[r] is None:
                return
            self._bind_out(out, _DeviceValue("product", seen[l].product(seen[r])))
        return self._start([l, r], body)

    def filter(self, i, fun: Callable, out):
        t = self.vars[i].type

        def body(seen):
            dom = self.odom if t == "lasp_orset" else self.gdom
            res = self._new_batch(t).filter(seen[i], dom.keep_bits(fun, self.cap))
            self._bind_out(out, _DeviceValue("canonical", res))
        return self._start([i], body)

    def map(self, i, fun: Callable, out):
        return self._seq_proc(i, out, lambda dom: SeqOutput.map(dom, fun))

    def fold(self, i, fun: Callable, out):
        return self._seq_proc(i, out, lambda dom: SeqOutput.fold(dom, fun))

    def _seq_proc(self, i, out, layout):
        t = self.vars[i].type

        def body(seen):
            dom = self.odom if t == "lasp_orset" else self.gdom
            so = layout(dom)
            res = self._batch_like(t, so.size).gather(seen[i], so.index())
            self._bind_out(out, _DeviceValue("seq", res, so))
        return self._start([i], body)


def _type_new(type_):
    """Type:new() (lasp_core.erl:339-346 substitutes it for an undefined threshold)."""
    if type_ == "lasp_orset_gbtree":
        from .gbtrees import empty
        return empty()
    return []


class _DeviceValue:
    __slots__ = ("rep", "batch", "seq")

    def __init__(self, rep, batch, seq=None):
        self.rep, self.batch, self.seq = rep, batch, seq


def _or_into(ctx, dst, a, b):
    """dst := a ⊔ b slot-wise for any representation: one k_or16 launch, or the
    per-actor max for G-Counters."""
    if isinstance(dst, engine.GCounterBatch):
        _lib.check(ctx.L.laspj_gcounter_join(ctx.h, dst.h, a.h, b.h), ctx.h)
    else:
        _lib.check(ctx.L.laspj_batch_join(ctx.h, dst.h, a.h, b.h), ctx.h)


def _concat_visible(dom: Domain, bits) -> list:
    return [dom.elements.terms[int(e)] for e in dom.elements.order()
            if (int(bits[int(e) >> 6]) >> (int(e) & 63)) & 1]

