"""Host side of the list-faithful values (include/laspj.h "list values").

A `ListSpace` keeps the device rank tables of one dictionary (codec.Domain): the term
order of every element slot (krank) and of every token slot (grank, 64 per element
slot), re-uploaded when the dictionary has grown.  `encode` / `decode` move a Lasp
value written as a Python term to and from the list items; `map_table`,
`filter_table` and `fold_table` evaluate a combinator's fun once per key (the NIF
would call the Erlang fun the same way) and hand the device its results.

Items (laspj.h): key = element slot, or LIST_PAIR | x << 31 | y for a product key
{X, Y}; token = 64*e + k (token slot k of element slot e), or LIST_COMPOUND | gx << 31
| gy for a product token [Tx, Ty]; bit 63 of a token = its flag.
"""

from __future__ import annotations

from typing import Callable, Optional

import numpy as np

from . import _lib
from .codec import CapacityError, Domain, NonCanonical
from .terms import term_cmp, term_key

PAIR = _lib.LIST_PAIR
COMPOUND = _lib.LIST_COMPOUND
REMOVED = _lib.LIST_REMOVED
ID = (1 << 31) - 1
FAILED = (1 << 64) - 1          # table entry of a key on which the fun raised


class FunFailed(RuntimeError):
    """The combinator's fun raised on a key of its input (the reference body crashes)."""


class ListSpace:
    """Rank tables of one Domain on one device context, kept up to date incrementally.

    krank (element slots) is dense: rank = position in the element order, rebuilt with
    one vectorised pass when the element dictionary grew.  grank (token ids g = 64 e + k)
    holds order LABELS, not dense ranks: the kernels only compare ranks and test them
    for equality (include/laspj.h "list values"), so a label strictly between its
    neighbours' labels serves as well as a rank.  A new token term takes the midpoint of
    the gap its neighbours leave (a term equal to a placed one takes that one's label),
    and only its grank entry is re-uploaded; when a gap is used up every distinct term
    is relabelled evenly over [1, 2^31) and the table re-uploaded whole.  An update/3
    that mints one token so costs a binary search and a 4-byte upload, not a rebuild of
    64 x (element slots) entries."""

    LABEL_END = 1 << 31              # labels are 31-bit (pairs pack two, laspj.h)
    LABEL_STEP = 1 << 16             # gap left after the last / before the first term

    def __init__(self, ctx, dom: Domain, tokens: bool = True):
        self.ctx, self.dom, self.tokens = ctx, dom, tokens
        self._order = _lib.ListOrder()
        self._kbuf = None
        self._kfor = None                 # the element order array krank was built from
        # token labels: the distinct token terms in term order (keys for bisect), their
        # labels, and the token ids g = 64 e + k carrying each
        self._tkeys: list = []
        self._tlab: list = []
        self._tids: list = []
        self._seen: dict = {}             # element slot -> tokens placed
        self._log_rank = 0                # position in dom.tok_log the labels have seen
        self._grank = np.zeros((0,), dtype=np.uint32)
        self._gbuf = None
        self._relabels = 0
        self._log_tord = 0                # position in dom.tok_log the token-order rows have seen
        # laspj_list_from_set's per-element token order rows, refreshed per element
        self._tord = np.zeros((0, 64), dtype=np.uint8)
        self._tord_buf = None
        self._eorder = None               # (elements order array, its device buffer)

    def order(self) -> _lib.ListOrder:
        """laspj_list_order over the current dictionary (brought up to date first)."""
        d = self.dom
        K = max(1, d.size)
        eord = d.elements.order()
        if self._kfor is not eord or self._order.nkeys != K:
            krank = np.zeros((K,), dtype=np.uint32)
            krank[eord] = np.arange(len(eord), dtype=np.uint32)
            if self._kbuf is None or self._kbuf.nbytes < krank.nbytes:
                self._kbuf = self.ctx.buffer(max(4, 2 * krank.nbytes))
            self._kbuf.upload(krank)
            self._order.krank = self._kbuf.h.value
            self._order.nkeys = K
            self._kfor = eord
        if self.tokens:
            self._place_tokens(K)
        else:
            self._order.grank = None
            self._order.ntokens = 0
        return self._order

    def _place_tokens(self, K: int):
        import bisect
        d = self.dom
        grow = 64 * K > len(self._grank)
        if grow:                                  # room for 64 x (twice the slots)
            g2 = np.zeros((64 * max(2 * K, 64),), dtype=np.uint32)
            g2[:len(self._grank)] = self._grank
            self._grank = g2
            self._gbuf = self.ctx.buffer(self._grank.nbytes)
        log = d.tok_log
        changed, relabel = [], False
        if len(log) - self._log_rank > max(4096, len(self._tkeys) // 8):
            # many new tokens (a first bind of a large value): one sort of every token
            grown = sorted(set(log[self._log_rank:]))
            self._log_rank = len(log)
            for e in grown:
                self._seen[e] = len(d.tokens[e].terms)
            allg = sorted(((term_key(t), 64 * e + k) for e in self._seen
                           for k, t in enumerate(d.tokens[e].terms[:min(self._seen[e], 64)])),
                          key=lambda x: x[0])
            self._tkeys, self._tids = [], []
            for key, g in allg:
                if self._tkeys and not (self._tkeys[-1] < key):
                    self._tids[-1].append(g)
                else:
                    self._tkeys.append(key)
                    self._tids.append([g])
            relabel = True
        elif self._log_rank < len(log):
            grown = sorted(set(log[self._log_rank:]))
            self._log_rank = len(log)
            for e in grown:
                terms = d.tokens[e].terms
                for k in range(self._seen.get(e, 0), min(len(terms), 64)):
                    key = term_key(terms[k])
                    g = 64 * e + k
                    i = bisect.bisect_left(self._tkeys, key)
                    if i < len(self._tkeys) and not (key < self._tkeys[i]) and \
                            not (self._tkeys[i] < key):
                        self._tids[i].append(g)        # an equal term: its label
                        self._grank[g] = self._tlab[i]
                        changed.append(g)
                        continue
                    lo = self._tlab[i - 1] if i > 0 else 0
                    hi = self._tlab[i] if i < len(self._tlab) else self.LABEL_END
                    if i == len(self._tlab):
                        lab = lo + min(self.LABEL_STEP, (hi - lo) // 2)
                    elif i == 0:
                        lab = hi - min(self.LABEL_STEP, (hi - lo) // 2)
                    else:
                        lab = (lo + hi) // 2
                    self._tkeys.insert(i, key)
                    self._tids.insert(i, [g])
                    if lo < lab < hi:
                        self._tlab.insert(i, lab)
                        self._grank[g] = lab
                        changed.append(g)
                    else:                              # the gap is used up
                        self._tlab.insert(i, lo)
                        relabel = True
                self._seen[e] = len(terms)
        if relabel:
            # evenly over the lower half, leaving the upper half for appended terms
            n = len(self._tkeys)
            step = (self.LABEL_END - 1) // (2 * n + 2)
            if step < 1:
                raise OverflowError("more than 2^31 distinct token terms")
            self._tlab = [step * (j + 1) for j in range(n)]
            lens = np.fromiter((len(x) for x in self._tids), dtype=np.int64, count=n)
            ids = np.fromiter((g for x in self._tids for g in x), dtype=np.int64,
                              count=int(lens.sum()))
            self._grank[ids] = np.repeat(np.asarray(self._tlab, dtype=np.uint32), lens)
            self._relabels += 1
        if grow or relabel or len(changed) > 4096:
            self._gbuf.upload(self._grank)
        else:
            for g in changed:
                self._gbuf.upload(self._grank[g:g + 1], offset=4 * g)
        self._order.grank = self._gbuf.h.value
        self._order.ntokens = 64 * K

    def set_orders(self, E: int):
        """(elem_order buffer, nslots, tok_order buffer) for laspj_list_from_set over a
        dense batch of E element slots; only the rows of elements whose token dictionary
        grew are rebuilt and re-uploaded."""
        d = self.dom
        order = d.elements.order()
        if self._eorder is None or self._eorder[0] is not order:
            o32 = order.astype(np.uint32)
            eb = self.ctx.buffer(max(4, o32.nbytes))
            if len(o32):
                eb.upload(o32)
            self._eorder = (order, eb)
        eb = self._eorder[1]
        tb = None
        if self.tokens:
            log = d.tok_log
            if self._tord.shape[0] != E:
                self._tord = np.full((E, 64), 0xFF, dtype=np.uint8)
                self._tord_buf = self.ctx.buffer(self._tord.nbytes)
                todo, whole = range(min(d.size, E)), True
            else:
                todo, whole = sorted(set(e for e in log[self._log_tord:] if e < E)), False
            self._log_tord = len(log)
            for e in todo:
                o = d.tokens[e].order()
                o = o[o < 64]
                self._tord[e, :] = 0xFF
                self._tord[e, :len(o)] = o
            if whole:
                self._tord_buf.upload(self._tord.reshape(-1))
            else:
                for e in todo:
                    self._tord_buf.upload(self._tord[e], offset=64 * e)
            tb = self._tord_buf
        return eb, len(order), tb


# ------------------------------------------------------------------- items <-> terms

def _key_item(dom: Domain, key, pairs: bool) -> int:
    if pairs and isinstance(key, tuple) and len(key) == 2:
        return PAIR | (dom.element_slot(key[0]) << 31) | dom.element_slot(key[1])
    return dom.element_slot(key)


def _key_term(dom: Domain, item: int):
    if item & PAIR:
        return (dom.elements.terms[(item >> 31) & ID], dom.elements.terms[item & ID])
    return dom.elements.terms[item & ID]


def _tok_term(dom: Domain, item: int):
    if item & COMPOUND:
        gx, gy = (item >> 31) & ID, item & ID
        return [dom.tokens[gx >> 6].terms[gx & 63], dom.tokens[gy >> 6].terms[gy & 63]]
    g = item & ID
    return dom.tokens[g >> 6].terms[g & 63]


def _tslot(dom: Domain, e: int, tok) -> int:
    """A token's slot as a list token id part: list values name 64 token slots per
    element (g = 64 e + k); a wide domain's later slots are not representable here."""
    k = dom.token_slot(e, tok)
    if k >= 64:
        raise CapacityError(f"element {dom.elements.terms[e]!r}: list values hold 64 "
                            f"tokens per element")
    return k


def encode(dom: Domain, term, gset: bool, pairs: bool = False):
    """A Lasp value (any list: orddict-shaped or not) -> (keys, toff, toks) items.
    With `pairs`, 2-tuple keys become product key items and, under them, 2-list tokens
    product token items (the shape product outputs have)."""
    if not isinstance(term, list):
        raise NonCanonical("a set value is a list")
    keys = np.zeros((len(term),), dtype=np.uint64)
    if gset:
        for i, e in enumerate(term):
            keys[i] = _key_item(dom, e, pairs)
        return keys, None, None
    toff = np.zeros((len(term) + 1,), dtype=np.uint32)
    toks = []
    for i, entry in enumerate(term):
        if not (isinstance(entry, tuple) and len(entry) == 2 and isinstance(entry[1], list)):
            raise NonCanonical(f"entry {entry!r} is not {{Key, [{{Token, Bool}}]}}")
        k, ts = entry
        item = _key_item(dom, k, pairs)
        keys[i] = item
        for t in ts:
            if not (isinstance(t, tuple) and len(t) == 2 and isinstance(t[1], bool)):
                raise NonCanonical(f"token entry {t!r} is not {{Token, Bool}}")
            tok, flag = t
            if item & PAIR and isinstance(tok, list) and len(tok) == 2:
                x, y = (item >> 31) & ID, item & ID
                g = COMPOUND | ((64 * x + _tslot(dom, x, tok[0])) << 31) | \
                    (64 * y + _tslot(dom, y, tok[1]))
            else:
                e = item & ID if not item & PAIR else None
                if e is None:
                    raise NonCanonical("a product key's tokens are [Tx, Ty] pairs")
                g = 64 * e + _tslot(dom, e, tok)
            toks.append(g | (REMOVED if flag else 0))
        toff[i + 1] = len(toks)
    return keys, toff, np.asarray(toks, dtype=np.uint64)


def decode(dom: Domain, keys, toff, toks, gset: bool) -> list:
    if gset:
        return [_key_term(dom, int(k)) for k in keys]
    out = []
    for i, k in enumerate(keys):
        run = toks[int(toff[i]):int(toff[i + 1])]
        out.append((_key_term(dom, int(k)),
                    [(_tok_term(dom, int(t)), bool(int(t) & REMOVED)) for t in run]))
    return out


# ------------------------------------------------------------------- fun tables

class FunCache:
    """Results of one combinator fun per key term (the fun is fixed for a process, so
    each key is evaluated once over the process's life)."""

    def __init__(self, fun: Callable):
        self.fun = fun
        self.cache = {}

    def __call__(self, x):
        from .terms import hkey
        k = hkey(x)
        if k not in self.cache:
            try:
                self.cache[k] = (True, self.fun(x))
            except Exception as e:           # the reference body would crash on x
                self.cache[k] = (False, e)
        return self.cache[k]


def _arg(term, gset: bool):
    """What the body passes to the fun, and the tail it re-attaches: lasp_core matches
    `{X, Causality}` before `X` (lasp_core.erl:467-474, 648-655, 688-695), so a G-Set
    element that is a 2-tuple goes through the OR-Set branch."""
    if gset and isinstance(term, tuple) and len(term) == 2:
        return term[0], (term[1],)
    return term, None


def map_table(dom: Domain, fun: FunCache, terms, gset: bool) -> np.ndarray:
    out = np.zeros((len(terms),), dtype=np.uint64)
    for i, t in enumerate(terms):
        x, tail = _arg(t, gset)
        ok, v = fun(x)
        if not ok:
            out[i] = FAILED
            continue
        out[i] = dom.element_slot(v if tail is None else (v,) + tail)
    return out


def filter_table(fun: FunCache, terms, gset: bool) -> np.ndarray:
    """keep = 1 when F(V) =:= true, V = the key (OR-Set) or the element (G-Set; its
    first component when it is a 2-tuple, lasp_core.erl:688-695); 2 when F raised."""
    out = np.zeros((len(terms),), dtype=np.uint8)
    for i, t in enumerate(terms):
        x = _arg(t, gset)[0]
        ok, v = fun(x)
        out[i] = 2 if not ok else (1 if v is True else 0)
    return out


def fold_table(dom: Domain, fun: FunCache, terms, gset: bool):
    off = np.zeros((len(terms) + 1,), dtype=np.uint32)
    keys = []
    for i, t in enumerate(terms):
        x, tail = _arg(t, gset)
        ok, v = fun(x)
        if ok and not isinstance(v, list):
            ok = False                       # a generator over a non-list crashes
        if not ok:
            keys.append(FAILED)
        else:
            keys.extend(dom.element_slot(y if tail is None else (y,) + tail) for y in v)
        off[i + 1] = len(keys)
    return off, np.asarray(keys, dtype=np.uint64)


def table_terms(dom: Domain, lst, pairs: bool):
    """(terms, per_entry): a table per element slot of the dictionary (no download);
    product outputs (pair keys) get one per entry of the list (its keys downloaded)."""
    if pairs:
        keys, _o, _t = lst.download()
        return [_key_term(dom, int(k)) for k in keys], True
    return list(dom.elements.terms), False
