"""OTP stdlib clauses used by the lattice layer — oracle restatement (TEST INFRASTRUCTURE).

The reference calls `orddict`, `ordsets`, `lists` and `sets` from OTP's stdlib, which
is a third-party dependency not vendored in the reference (rebar.config:3-12 pins no OTP;
the code era is OTP R16/17).  The clauses below restate OTP 17's
published `orddict.erl` / `ordsets.erl` / `lists.erl` / `sets.erl` behaviour exactly as
written — including what they do on unsorted or duplicated input, which the
reference's combinators produce — as iterative loops so that
10^4..10^5-element lists do not hit Python's recursion limit.

Comparisons use Erlang term order (terms.compare: `<`, `>`, and `==` for the
fall-through clause); `lists:member` and `sets` use exact matching (`=:=`).
"""

from __future__ import annotations

from .terms import compare, exact_eq, Key, _rank, _atom_name

# ----------------------------------------------------------------------------- orddict


def orddict_new():
    return []


def orddict_find(key, d):
    """orddict:find/2 — early exit at the first key greater than `key` (even if the
    list is unsorted)."""
    for k, v in d:
        c = compare(key, k)
        if c < 0:
            return None
        if c == 0:
            return ("ok", v)
    return None


def orddict_store(key, new, d):
    """orddict:store/3:
    store(K,N,[{K1,_}=E|D]) when K<K1 -> [{K,N},E|D];
    store(K,N,[{K1,_}=E|D]) when K>K1 -> [E|store(K,N,D)];
    store(K,N,[{_,_}|D])              -> [{K,N}|D];
    store(K,N,[])                     -> [{K,N}]."""
    out = []
    for i, (k, v) in enumerate(d):
        c = compare(key, k)
        if c < 0:
            out.append((key, new))
            out.extend(d[i:])
            return out
        if c == 0:
            out.append((key, new))
            out.extend(d[i + 1:])
            return out
        out.append((k, v))
    out.append((key, new))
    return out


def orddict_merge(fun, d1, d2):
    """orddict:merge/3 — a pure two-finger merge (reproduced as written on
    non-canonical input):
    merge(F,[{K1,_}=E1|D1],[{K2,_}=E2|D2]) when K1<K2 -> [E1|merge(F,D1,[E2|D2])];
    merge(F,[{K1,_}=E1|D1],[{K2,_}=E2|D2]) when K1>K2 -> [E2|merge(F,[E1|D1],D2)];
    merge(F,[{K1,V1}|D1],[{_,V2}|D2]) -> [{K1,F(K1,V1,V2)}|merge(F,D1,D2)];
    merge(F,[],D2) -> D2;   merge(F,D1,[]) -> D1."""
    out = []
    i = j = 0
    n1, n2 = len(d1), len(d2)
    while i < n1 and j < n2:
        k1, v1 = d1[i]
        k2, v2 = d2[j]
        c = compare(k1, k2)
        if c < 0:
            out.append(d1[i])
            i += 1
        elif c > 0:
            out.append(d2[j])
            j += 1
        else:
            out.append((k1, fun(k1, v1, v2)))
            i += 1
            j += 1
    if i < n1:
        out.extend(d1[i:])
    if j < n2:
        out.extend(d2[j:])
    return out


def orddict_filter(pred, d):
    """orddict:filter/2 — order preserving; the predicate must return a boolean."""
    out = []
    for k, v in d:
        r = pred(k, v)
        if r is True:
            out.append((k, v))
        elif r is not False:
            raise ValueError("case_clause: orddict:filter predicate returned a non-boolean")
    return out


def orddict_fetch_keys(d):
    return [k for k, _ in d]


def orddict_fold(fun, acc, d):
    for k, v in d:
        acc = fun(k, v, acc)
    return acc


def orddict_size(d):
    return len(d)


def orddict_to_list(d):
    return list(d)


# ----------------------------------------------------------------------------- ordsets


def ordsets_new():
    return []


def ordsets_union(s1, s2):
    """ordsets:union/2 as in OTP 17 (note the argument switch in clause 2):
    union([E1|Es1],[E2|_]=S2) when E1<E2 -> [E1|union(Es1,S2)];
    union([E1|_]=S1,[E2|Es2]) when E1>E2 -> [E2|union(Es2,S1)];   % switch arguments!
    union([E1|Es1],[_E2|Es2])           -> [E1|union(Es1,Es2)];
    union([],Es2) -> Es2;  union(Es1,[]) -> Es1.
    Identical to a plain two-finger merge on canonical sets; differs only in which of
    two `==`-equal terms survives and on non-canonical input (parity unpinned there)."""
    a, b = s1, s2
    i = j = 0
    out = []
    while i < len(a) and j < len(b):
        c = compare(a[i], b[j])
        if c < 0:
            out.append(a[i])
            i += 1
        elif c > 0:
            out.append(b[j])
            # switch arguments: union(Es2, Set1)
            a, b, i, j = b, a, j + 1, i
        else:
            out.append(a[i])
            i += 1
            j += 1
    if i >= len(a):
        out.extend(b[j:])
    else:
        out.extend(a[i:])
    return out


def ordsets_add_element(e, s):
    """add_element(E,[H|Es]) when E>H -> [H|add_element(E,Es)];
    add_element(E,[H|_]=Set) when E<H -> [E|Set];
    add_element(_E,[_H|_]=Set) -> Set;   add_element(E,[]) -> [E]."""
    for i, h in enumerate(s):
        c = compare(e, h)
        if c < 0:
            return list(s[:i]) + [e] + list(s[i:])
        if c == 0:
            return list(s)
    return list(s) + [e]


def ordsets_to_list(s):
    return list(s)


def ordsets_from_list(lst):
    return lists_usort(lst)


def ordsets_fold(fun, acc, s):
    for e in s:
        acc = fun(e, acc)
    return acc


# ----------------------------------------------------------------------------- lists


def lists_sort(lst):
    """lists:sort/1 — stable sort by term order."""
    return sorted(lst, key=Key)


def lists_usort(lst):
    """lists:usort/1 — sort, keeping only the first of `==`-equal elements."""
    out = []
    for e in sorted(lst, key=Key):
        if out and compare(out[-1], e) == 0:
            continue
        out.append(e)
    return out


def lists_keyfind(key, lst):
    """lists:keyfind(Key, 1, List): first tuple whose first element `==` Key."""
    for t in lst:
        if isinstance(t, tuple) and len(t) >= 1 and compare(t[0], key) == 0:
            return t
    return False


def lists_member(e, lst):
    """lists:member/2 uses exact matching (=:=)."""
    return any(exact_eq(e, x) for x in lst)


# ----------------------------------------------------------------------------- sets
# OTP `sets` match elements exactly (=:=).  A hashable canonical form stands in for
# the hash buckets; only membership semantics matter on this path.


def exact_key(t):
    r = _rank(t)
    if r == 0:
        return ("f" if isinstance(t, float) else "i", t)
    if r == 1:
        return ("a", _atom_name(t))
    if r == 10:
        return ("b", bytes(t))
    if r == 6:
        return ("t",) + tuple(exact_key(x) for x in t)
    if r in (8, 9):
        return ("l",) + tuple(exact_key(x) for x in t)
    raise TypeError(t)


def sets_from_list(lst):
    return {exact_key(e): e for e in lst}


def sets_is_subset(s1, s2) -> bool:
    return all(k in s2 for k in s1)
