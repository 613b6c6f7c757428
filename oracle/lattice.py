"""lasp_lattice restatement (orset / orset_gbtree / gset / gcounter clauses) — oracle (TEST INFRASTRUCTURE).

Follows src/lasp_lattice.erl.  `prev` / `cur` are full lattice states (not values).
"""

from __future__ import annotations

from . import gbtrees as gb, otp, gset as _gset


def threshold_met(type_, value, threshold) -> bool:
    """threshold_met/3 — lasp_lattice.erl:62-75 (gset / orset) and :87-90 (gcounter)."""
    strict = isinstance(threshold, tuple) and len(threshold) == 2 and threshold[0] == "strict"
    if type_ == "riak_dt_gcounter":
        # Erlang term order: numbers compare numerically, anything else is above them
        from .terms import compare
        v = gcounter_value(value)
        return compare(threshold[1], v) < 0 if strict else compare(threshold, v) <= 0
    if strict:
        return is_strict_inflation(type_, threshold[1], value)
    return is_inflation(type_, threshold, value)


def is_inflation(type_, prev, cur) -> bool:
    """is_inflation/3 -> is_lattice_inflation/3 — lasp_lattice.erl:97-98."""
    if type_ == "lasp_gset":
        # :137-140
        return otp.sets_is_subset(otp.sets_from_list(_gset.value(prev)),
                                  otp.sets_from_list(_gset.value(cur)))
    if type_ == "lasp_orset":
        # :153-161 — every Prev element found in Cur (lists:keyfind, ==) and its ids
        # inflated; removed flags are ignored.
        acc = True
        for elem, ids in prev:
            found = otp.lists_keyfind(elem, cur)
            if found is False:
                acc = acc and False
            else:
                acc = acc and _ids_inflated(ids, found[1])
        return acc
    if type_ == "lasp_orset_gbtree":
        # :142-150 — in-order fold over Prev; gb_trees:lookup (==) in Cur; ids
        # inflated per ids_inflated(lasp_orset_gbtree, ...) :287-295
        acc = True
        for elem, ids in gb.to_list(prev):
            found = gb.lookup(elem, cur)
            if found is None:
                acc = acc and False
            else:
                acc = acc and all(gb.lookup(t, found[1]) is not None
                                  for t, _ in gb.to_list(ids))
        return acc
    if type_ == "riak_dt_gcounter":
        # :169-179
        acc = True
        cur_l = otp.lists_sort(list(cur))
        for actor, count in otp.lists_sort(list(prev)):
            found = otp.lists_keyfind(actor, cur_l)
            acc = acc and (found is not False and count <= found[1])
        return acc
    raise ValueError(f"type not on this path: {type_}")


def _ids_inflated(prev_ids, cur_ids) -> bool:
    """ids_inflated(lasp_orset, ...) — lasp_lattice.erl:277-285."""
    acc = True
    for tok, _ in prev_ids:
        acc = acc and (otp.lists_keyfind(tok, cur_ids) is not False)
    return acc


def is_strict_inflation(type_, prev, cur) -> bool:
    """is_strict_inflation/3 -> is_lattice_strict_inflation/3 — lasp_lattice.erl:105-106."""
    if type_ == "lasp_gset":
        # :212-215
        return is_inflation(type_, prev, cur) and not _term_eq(
            otp.lists_usort(_gset.value(prev)), otp.lists_usort(_gset.value(cur)))
    if type_ == "lasp_orset_gbtree":
        # :217-233 — no `[]` special case; `Ids =/= Ids1` compares the token TREES
        # (shape included); new elements by gb_trees:size
        infl = is_inflation(type_, prev, cur)
        deleted = False
        for elem, ids in gb.to_list(prev):
            found = gb.lookup(elem, cur)
            if found is not None:
                deleted = deleted or not gb.structurally_equal(ids, found[1])
        return infl and (deleted or gb.size(prev) < gb.size(cur))
    if type_ == "lasp_orset":
        # :235-253
        if prev == [] and cur != []:
            return True
        infl = is_inflation(type_, prev, cur)
        deleted = False
        for elem, ids in prev:
            found = otp.lists_keyfind(elem, cur)
            if found is not False:
                deleted = deleted or not _term_eq(_tok_term(ids), _tok_term(found[1]))
        new_elems = len(prev) < len(cur)
        return infl and (deleted or new_elems)
    if type_ == "riak_dt_gcounter":
        # :273-275
        return gcounter_value(prev) < gcounter_value(cur)
    raise ValueError(f"type not on this path: {type_}")


def orset_causal_product(xs, ys):
    """orset_causal_product/2 — lasp_lattice.erl:303-308: fully reversed foldl, so
    the token list comes out descending for sorted inputs."""
    x_acc = []
    for x, x_del in xs:
        y_acc = []
        for y, y_del in ys:
            y_acc = [([x, y], x_del or y_del)] + y_acc
        x_acc = y_acc + x_acc
    return x_acc


def orset_causal_union(xs, ys):
    """orset_causal_union/2 — lasp_lattice.erl:311-312."""
    return list(xs) + list(ys)


def gcounter_value(c) -> int:
    """riak_dt_gcounter:value/1 — sum of per-actor counts (orddict Actor -> Count)."""
    return sum(n for _a, n in c)


def _tok_term(ids):
    return [(t, r) for t, r in ids]


def _term_eq(a, b) -> bool:
    from .terms import exact_eq
    # `=/=` in the reference is exact inequality
    return exact_eq(a, b)
