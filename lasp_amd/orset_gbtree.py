"""lasp_orset_gbtree mirror over the MI355X engine (src/lasp_orset_gbtree.erl).

`lasp_orset_gbtree` is Lasp's default set for internal state (`?SET`,
include/lasp.hrl:30): the same observed-remove set as lasp_orset with the two
orddict levels replaced by gb_trees (Elem -> gb_tree Token -> Removed).  Its contents
map onto the same columnar cells ({p, r} per element slot), so every call runs on the
same HIP kernels as lasp_orset; only the host-side term walk differs:

* operands are walked in order (gb_trees:to_list/1) into the shared Domain;
* results are built as the trees OTP builds for them — `gb_trees_ext:merge/3`
  inserts keys in ascending order into `empty()` (the outer tree, and the token tree of
  an element both operands hold; an element of one operand keeps its token tree as it
  is), and so does remove_elem's rebuild, which `lasp_amd.gbtrees.build_sorted`
  reproduces; update/3
  replays its gb_trees:insert / enter calls on the operand's own trees
  (lasp_amd.gbtrees.insert / enter), so an update-built tree keeps the shape its
  insertion history gives it.  Only keys are placed on the host: the values come, in
  order, from the device's result.

Semantics kept from the reference:
* add / add_by_token insert the token with gb_trees:insert/3 (:232-240): a token that
  is already present raises {key_exists, Token} (`KeyExists`), detected on the device
  (LASPJ_OP_INSERT / LASPJ_OPST_KEY_EXISTS) with the call left unapplied;
* remove of an absent element -> {error, {precondition, {not_present, E}}};
* value/1 and value(removed) are in-order folds (:67-76, :93-101).
* equal/2 is gb_trees_ext:equal: in-order {Key, Value} matches, where Value is the
  inner token TREE, so inner shapes count — the device compares contents, the host the
  inner trees' shapes; strict inflation (lasp_lattice.erl:217-233) likewise counts an
  element whose token tree changed shape as changed (lasp_amd.lattice).
"""

from __future__ import annotations

import os
from typing import List, Sequence, Tuple

import numpy as np

from . import _lib, gbtrees as gbt
from .codec import Domain
from .orset import _batch, _waste_pct, context
from .terms import Atom


class KeyExists(Exception):
    """erlang:error({key_exists, Token}) raised by gb_trees:insert/3 in add_elem."""

    def __init__(self, token):
        super().__init__(("key_exists", token))
        self.token = token


def to_orddict(s) -> list:
    """Both levels walked in order: the orddict-shaped contents of the set."""
    out = []
    for elem, toks in gbt.walk(s):
        pairs = gbt.walk(toks)
        for _t, rm in pairs:
            if not isinstance(rm, bool):
                raise ValueError(f"badarg: token flag {rm!r}")
        out.append((elem, pairs))
    return out


def from_orddict(od) -> tuple:
    """The tree gb_trees_ext:merge builds for these contents."""
    return gbt.build_sorted([(e, gbt.build_sorted(toks)) for e, toks in od])


# --------------------------------------------------------------------------- API

def new():
    """new/0 — src/lasp_orset_gbtree.erl:63-65."""
    return gbt.empty()


def merge(a, b):
    """merge/2 — :134-140 (device join)."""
    return merge_many([(a, b)])[0]


def merge_many(pairs: Sequence[Tuple[tuple, tuple]]) -> List[tuple]:
    """merge/2 over many independent pairs in one launch."""
    if not pairs:
        return []
    dom = Domain()
    ods = [(to_orddict(a), to_orddict(b)) for a, b in pairs]
    A, E = _batch(dom, [p[0] for p in ods])
    B, _ = _batch(dom, [p[1] for p in ods])
    if B.elements != E:
        A, E = _batch(dom, [p[0] for p in ods])
    C = context().orset_batch(len(pairs), E)
    C.join(A, B)
    out = C.download()
    return [_merge_shape(a, b, dom.decode_orset(out[i])) for i, (a, b) in enumerate(pairs)]


def _merge_shape(a, b, od) -> tuple:
    """The tree gb_trees_ext:merge/3 builds (src/gb_trees_ext.erl:28-57) for the merged
    contents od: the outer tree by ascending inserts into empty(); an element in both
    operands gets its merged token tree (ascending inserts again); an element of one
    operand keeps that operand's token tree as it is (do_merge inserts Val1 / Val2
    itself) — its shape from the operand, its values from the device."""
    inner = []
    for elem, toks in od:
        ta, tb = gbt.lookup(elem, a), gbt.lookup(elem, b)
        if ta is not None and tb is not None:
            inner.append((elem, gbt.build_sorted(toks)))
        else:
            inner.append((elem, gbt.fill(ta if ta is not None else tb, [f for _t, f in toks])))
    return gbt.build_sorted(inner)


def value(s):
    """value/1 — :67-76 (device value bitmap, in-order)."""
    dom = Domain()
    b, _ = _batch(dom, [to_orddict(s)])
    return dom.decode_value_bits(b.value_bits()[0])


def value2(query, s):
    """value/2 — :78-104.  `{tokens, E}` is E's token tree (or empty()); since that is
    never the list `[]`, `{fragment, E}` is always the one-entry tree {E, Tokens}."""
    if isinstance(query, tuple) and len(query) == 2 and query[0] == "fragment":
        toks = value2(("tokens", query[1]), s)
        return gbt.insert(query[1], toks, gbt.empty())      # enter into empty()
    if isinstance(query, tuple) and len(query) == 2 and query[0] == "tokens":
        # gb_trees:get(Elem, ORSet): the element's own token tree — its shape from the
        # operand, its flags from the device's cell
        dom = Domain()
        b, _ = _batch(dom, [to_orddict(s)])
        es = dom.element_slot(query[1], create=False)
        tree = gbt.lookup(query[1], s)
        if es < 0 or tree is None:
            return gbt.empty()
        cell = b.fragment(es)[0]
        p, r = int(cell[0]), int(cell[1])
        td = dom.tokens[es]
        flags = [bool((r >> int(k)) & 1) for k in td.order() if (p >> int(k)) & 1]
        return gbt.fill(tree, flags)
    if query == "removed":
        dom = Domain()
        b, _ = _batch(dom, [to_orddict(s)])
        return dom.decode_value_bits(b.value_bits(removed=True)[0])
    return value(s)


def _unique(_actor) -> bytes:
    """unique/1 — :276-277: 20 random bytes."""
    return os.urandom(20)


def _compile(op, dom: Domain, ops: list, new_call: bool, script: list = None) -> None:
    """ops for the device; script = the (add | remove, elem, token) calls in order, for
    the shape replay"""
    if script is None:
        script = []
    kind = op[0]
    flag = _lib.OP_FLAG_NEW_CALL if new_call else 0
    if kind in ("add", "add_by_token"):
        elem = op[1] if kind == "add" else op[2]
        tok = _unique(None) if kind == "add" else op[1]
        es = dom.element_slot(elem)
        ops.append((0, es, _lib.OP_INSERT, dom.token_slot(es, tok), flag))
        script.append(("add", elem, tok))
    elif kind == "add_all":
        # foldl of `{ok, _} = update({add, E})` (:112-117): one call, fresh tokens
        for k, e in enumerate(op[1]):
            es = dom.element_slot(e)
            tok = _unique(None)
            ops.append((0, es, _lib.OP_INSERT, dom.token_slot(es, tok), flag if k == 0 else 0))
            script.append(("add", e, tok))
    elif kind == "remove":
        ops.append((0, dom.element_slot(op[1]), _lib.OP_REMOVE, 0, flag))
        script.append(("remove", op[1], None))
    elif kind == "remove_all":
        for k, e in enumerate(op[1]):           # remove_elems/2 (:255-263)
            ops.append((0, dom.element_slot(e), _lib.OP_REMOVE, 0, flag if k == 0 else 0))
            script.append(("remove", e, None))
    elif kind == "update":
        first = len(ops)                        # apply_ops/3 (:266-274)
        for sub in op[1]:
            _compile(sub, dom, ops, new_call=False, script=script)
        for j in range(first, len(ops)):
            r, e, k, sl, _f = ops[j]
            ops[j] = (r, e, k, sl, flag if j == first else 0)
    else:
        raise ValueError(f"function_clause: {op!r}")


def _replay(script, s):
    """The keys of the tree the reference's update calls build from s: add_elem inserts
    the token into the element's token tree and enters the element (:231-240),
    remove_elem re-enters every token into empty() in order (:242-253).  Values are
    placeholders (filled from the device)."""
    t = s
    for kind, elem, tok in script:
        inner = gbt.lookup(elem, t)
        if kind == "add":
            t = gbt.enter(elem, gbt.insert(tok, None, inner if inner is not None
                                           else gbt.empty()), t)
        else:
            t = gbt.update(elem, gbt.build_sorted([(k, None) for k in gbt.keys(inner)]), t)
    return t


def shape_info(t):
    """(outer canonical, {hkey(elem): token tree} for the elements whose token tree is
    not the ascending-insert shape, {hkey(elem)}) — what a store keeps of a value's
    shape besides its contents."""
    from .terms import hkey
    pairs = gbt.walk(t)
    outer = gbt.shape(t) == gbt.shape(gbt.build_sorted([(k, None) for k, _v in pairs]))
    odd = {}
    for e, inner in pairs:
        ks = gbt.keys(inner)
        if gbt.shape(inner) != gbt.shape(gbt.build_sorted([(k, None) for k in ks])):
            odd[hkey(e)] = inner
    return outer, odd, {hkey(e) for e, _v in pairs}


def with_shapes(od, odd) -> tuple:
    """The tree of the orddict od whose outer tree is ascending-insert shaped and whose
    token trees are too, except those named in odd (hkey -> a tree of the same keys)."""
    from .terms import hkey
    inner = []
    for e, toks in od:
        t = odd.get(hkey(e))
        inner.append((e, gbt.fill(t, [f for _t, f in toks]) if t is not None
                      else gbt.build_sorted(toks)))
    return gbt.build_sorted(inner)


def _with_values(t, od) -> tuple:
    """t's keys at both levels, its values from the orddict od (same keys, in order)."""
    if len(gbt.keys(t)) != len(od):
        raise ValueError("device contents and tree keys disagree")
    inner = []
    for (elem, toks), (_e, tree) in zip(od, gbt.walk(t)):
        inner.append(gbt.fill(tree, [f for _t, f in toks]))
    return gbt.fill(t, inner)


def update(op, actor, s):
    """update/3 — :106-124.  ("ok", S1) | ("error", ("precondition", ("not_present",
    E))); raises KeyExists where the reference's gb_trees:insert/3 crashes.  Contents
    and preconditions on the device; the returned trees have the shapes the
    reference's insert / enter sequence gives them."""
    od = to_orddict(s)
    dom = Domain()
    dom.register_orset(od)
    ops, script = [], []
    _compile(op, dom, ops, new_call=True, script=script)
    E = max(1, dom.size)
    b = context().orset_batch(1, E)
    b.upload(dom.encode_orset([od], E))
    st = b.apply_ops(ops)
    bad = np.nonzero((st == _lib.OPST_NOT_PRESENT) | (st == _lib.OPST_KEY_EXISTS))[0]
    if len(bad):
        r, es, _k, slot, _f = ops[int(bad[0])]
        if st[bad[0]] == _lib.OPST_KEY_EXISTS:
            raise KeyExists(dom.tokens[es].terms[slot])
        return ("error", ("precondition", ("not_present", dom.elements.terms[es])))
    return ("ok", _with_values(_replay(script, s), dom.decode_orset(b.download()[0])))


def update4(op, actor, s, _ctx=None):
    """update/4 — :126-128 (context ignored)."""
    return update(op, actor, s)


def equal(a, b) -> bool:
    """equal/2 — :142-144, gb_trees_ext:equal (src/gb_trees_ext.erl:59-68): in-order
    {Key, Value} pairs match, Value being the inner token tree — contents compared on
    the device, the inner trees' shapes on the host."""
    dom = Domain()
    oa, ob = to_orddict(a), to_orddict(b)
    dom.register_orset(oa)
    dom.register_orset(ob)
    E = max(1, dom.size)
    A = context().orset_batch(1, E)
    B = context().orset_batch(1, E)
    A.upload(dom.encode_orset([oa], E))
    B.upload(dom.encode_orset([ob], E))
    if not bool(A.equal(B)[0]):
        return False
    return all(gbt.shape(x) == gbt.shape(y)
               for (_e, x), (_f, y) in zip(gbt.walk(a), gbt.walk(b)))


def shapes_differ(prev, cur) -> bool:
    """Some element of prev found in cur (gb_trees:lookup) has a token tree of another
    shape — one half of `Ids =/= Ids1` in the strict-inflation clause
    (lasp_lattice.erl:217-233); the device compares the contents."""
    for elem, toks in gbt.walk(prev):
        other = gbt.lookup(elem, cur)
        if other is not None and gbt.shape(other) != gbt.shape(toks):
            return True
    return False


def precondition_context(s):
    """precondition_context/1 — :153-162 with minimum_tokens (:279-287): the device
    keeps the tokens flagged false; as in the reference, each element's value is the
    LIST [{Token, false}] minimum_tokens returns, entered in order into empty()."""
    dom = Domain()
    b, E = _batch(dom, [to_orddict(s)])
    out = context().orset_batch(1, E).precondition_context(b)
    return gbt.build_sorted(dom.decode_orset(out.download()[0]))


def stats(s):
    """stats/1 — :164-169 (element_count = gb_trees:size = elements with a token)."""
    dom = Domain()
    b, _ = _batch(dom, [to_orddict(s)])
    elems, adds, rems = (int(x) for x in b.stats()[0])
    return [("element_count", elems), ("adds_count", adds), ("removes_count", rems),
            ("waste_pct", _waste_pct(adds, rems))]


def stat(name, s):
    """stat/2 — :171-200 (unknown stat -> undefined)."""
    for k, v in stats(s):
        if k == name:
            return v
    return Atom("undefined")


def parent_clock(_clock, s):
    """parent_clock/2 — :130-132."""
    return s


def to_version(_version, s):
    """to_version/2 — :226-228."""
    return s
