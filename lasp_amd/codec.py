"""Dictionaries and the orddict <-> columnar codec (host side of the boundary).

The device never sees terms.  A `Domain` owns
  * the element dictionary: element term -> element slot (append-only), and
  * one token dictionary per element slot: token term -> token slot 0..63 (append-only).
Every batch of a domain uses those slots, so joins / predicates / combinators between
its batches are pure bit operations.  Slots are assigned in first-seen order; the
term order needed for decoding (orddict keys and token keys ascend in Erlang term
order) is a per-dictionary permutation cached on the host.

Canonical states only: the device layout expresses an orddict whose keys are unique
and ascending, whose token lists are unique, ascending and non-empty — which is every
state lasp_orset:new/update/merge can produce (lasp_orset.erl:63-134).  Anything else
(the unsorted / duplicated outputs of the map and fold combinators, SURVEY.md
Appendix B) raises NonCanonical instead of being silently canonicalised.
"""

from __future__ import annotations

from typing import Dict, Iterable, List, Sequence

import numpy as np

from .terms import hkey, same_term, term_cmp, term_key

TOKEN_SLOTS = 64


class NonCanonical(ValueError):
    """The orddict is not expressible in the columnar layout (see module doc)."""


class CapacityError(ValueError):
    """An element needs more than 64 token slots, or the batch has too few slots."""


class EqualTerms(CapacityError):
    """A term `==` to one that holds a slot but not `=:=` to it (1 and 1.0, {a, 1} and
    {a, 1.0}): orddict:merge / ordsets:union treat them as one key,
    so neither "first seen wins" nor a second slot gives the reference's answers — the
    value is not representable here (the store raises Unsupported)."""


class _Dict:
    def __init__(self, cap: int):
        self.cap = cap
        self.terms: List = []
        self.index: Dict = {}
        self._order = None
        self._skeys: List = []        # term_key of the placed slots, ascending

    def __len__(self):
        return len(self.terms)

    def slot(self, term, create: bool = True) -> int:
        k = hkey(term)
        s = self.index.get(k)
        if s is not None and not same_term(self.terms[s], term):
            raise EqualTerms(f"{term!r} == {self.terms[s]!r} but is another term")
        if s is None:
            if not create:
                return -1
            if len(self.terms) >= self.cap:
                raise CapacityError(f"dictionary full ({self.cap} slots)")
            s = len(self.terms)
            self.terms.append(term)
            self.index[k] = s
        return s

    def order(self) -> np.ndarray:
        """Slots in ascending term order (ties — `==`-equal terms — in slot order).  A
        dictionary that grew by a few terms places them by binary search (one new array
        per change, so callers may test it by identity); a large growth re-sorts."""
        n0 = 0 if self._order is None else len(self._order)
        n = len(self.terms)
        if n0 == n and self._order is not None:
            return self._order
        if n - n0 > 1024 or self._order is None:
            idx = sorted(range(n), key=lambda i: term_key(self.terms[i]))
            self._skeys = [term_key(self.terms[i]) for i in idx]
            self._order = np.asarray(idx, dtype=np.int64)
            return self._order
        import bisect
        # each new slot's place among the OLD keys (after its equals: ties stay in slot
        # order), then inserted together, last place first
        new = sorted((bisect.bisect_right(self._skeys, term_key(self.terms[i])),
                      term_key(self.terms[i]), i) for i in range(n0, n))
        for p, key, _i in reversed(new):
            self._skeys.insert(p, key)
        self._order = np.insert(self._order, [p for p, _k, _i in new], [i for _p, _k, i in new])
        return self._order

    def truncate(self, n: int) -> None:
        """Forget the slots from n on (an encode that failed part way: its registrations
        are undone, so a rejected value leaves no slots behind)."""
        if n >= len(self.terms):
            return
        for t in self.terms[n:]:
            self.index.pop(hkey(t), None)
        del self.terms[n:]
        if self._order is not None and len(self._order) > n:
            self._order, self._skeys = None, []


class Domain:
    """Element + token dictionaries shared by all batches of one engine domain."""

    def __init__(self, element_capacity: int = 1 << 30, token_capacity: int = TOKEN_SLOTS):
        self.elements = _Dict(element_capacity)
        self.token_capacity = token_capacity      # token slots per element (64 k when wide)
        self.tokens: List[_Dict] = []
        # element slots in the order their token dictionaries gained a slot (one entry
        # per new token): readers keep a position in it to update what they derived
        self.tok_log: List[int] = []

    def element_slot(self, elem, create: bool = True) -> int:
        s = self.elements.slot(elem, create)
        while create and len(self.tokens) < len(self.elements):
            self.tokens.append(_Dict(self.token_capacity))
        return s

    def token_slot(self, eslot: int, tok, create: bool = True) -> int:
        try:
            td = self.tokens[eslot]
            n = len(td.terms)
            s = td.slot(tok, create)
            if len(td.terms) != n:
                self.tok_log.append(eslot)
            return s
        except EqualTerms:
            raise
        except CapacityError as e:
            raise CapacityError(f"element {self.elements.terms[eslot]!r} has more than "
                                f"{self.token_capacity} tokens") from e

    @property
    def size(self) -> int:
        return len(self.elements)

    def journal(self) -> "_Journal":
        """`with dom.journal(): ...` — registrations made inside the block are undone
        when it raises (the device store commits slots only for values it encodes)."""
        return _Journal(self)

    # ------------------------------------------------------------------ OR-Set
    def register_orset(self, s) -> None:
        for elem, toks in s:
            es = self.element_slot(elem)
            for tok, _rm in toks:
                self.token_slot(es, tok)

    def encode_orset(self, states: Sequence, E: int) -> np.ndarray:
        """orddicts -> (len(states), E, 2) uint64 {p, r} cells."""
        for s in states:
            self.register_orset(s)
        if self.size > E:
            raise CapacityError(f"{self.size} elements do not fit {E} slots")
        out = np.zeros((len(states), E, 2), dtype=np.uint64)
        for i, s in enumerate(states):
            _check_canonical_orset(s)
            for elem, toks in s:
                es = self.element_slot(elem, create=False)
                p = r = 0
                for tok, rm in toks:
                    t = self.token_slot(es, tok, create=False)
                    if t >= 64:
                        raise CapacityError(f"element {elem!r}: token slot {t} needs wide cells")
                    bit = 1 << t
                    p |= bit
                    if rm is True:
                        r |= bit
                    elif rm is not False:
                        raise NonCanonical(f"token flag {rm!r} is not a boolean")
                out[i, es, 0] = p
                out[i, es, 1] = r
        return out

    def token_words(self) -> int:
        """{p, r} pairs a cell needs for the widest element's token slots (1: narrow)."""
        most = max((len(t) for t in self.tokens), default=0)
        return max(1, (most + 63) // 64)

    def orset_words(self, states: Sequence) -> int:
        """{p, r} pairs per cell the states' own token slots need (registering them):
        1 when every token slot they hold is < 64."""
        most = -1
        for s in states:
            for elem, toks in s:
                es = self.element_slot(elem)
                for tok, _rm in toks:
                    most = max(most, self.token_slot(es, tok))
        return max(1, (most + 64) // 64)

    def encode_orset_wide(self, states: Sequence, E: int, k: int) -> np.ndarray:
        """orddicts -> (len(states), E, k, 2) uint64 {p, r} pairs (LASPJ_KIND_ORSET_WIDE):
        token slot t in pair t // 64, bit t % 64."""
        for s in states:
            self.register_orset(s)
        if self.size > E:
            raise CapacityError(f"{self.size} elements do not fit {E} slots")
        out = np.zeros((len(states), E, k, 2), dtype=np.uint64)
        for i, s in enumerate(states):
            _check_canonical_orset(s)
            for elem, toks in s:
                es = self.element_slot(elem, create=False)
                for tok, rm in toks:
                    t = self.token_slot(es, tok, create=False)
                    if t // 64 >= k:
                        raise CapacityError(f"token slot {t} needs more than {k} words")
                    bit = np.uint64(1 << (t % 64))
                    out[i, es, t // 64, 0] |= bit
                    if rm is True:
                        out[i, es, t // 64, 1] |= bit
                    elif rm is not False:
                        raise NonCanonical(f"token flag {rm!r} is not a boolean")
        return out

    def decode_orset_wide(self, cells: np.ndarray) -> list:
        """(E, k, 2) pairs -> orddict (keys and tokens ascending in term order)."""
        out = []
        k = cells.shape[1]
        for es in self.elements.order():
            if es >= cells.shape[0]:
                continue
            ps = [int(cells[es, j, 0]) for j in range(k)]
            if not any(ps):
                continue
            rs = [int(cells[es, j, 1]) for j in range(k)]
            td = self.tokens[es]
            toks = [(td.terms[t], bool((rs[t // 64] >> (t % 64)) & 1))
                    for t in (int(x) for x in td.order())
                    if t < 64 * k and (ps[t // 64] >> (t % 64)) & 1]
            out.append((self.elements.terms[es], toks))
        return out

    def decode_orset(self, cells: np.ndarray) -> list:
        """(E, 2) cells -> orddict (keys and tokens ascending in term order)."""
        out = []
        p_col = cells[:, 0]
        for es in self.elements.order():
            if es >= cells.shape[0]:
                continue
            p = int(p_col[es])
            if not p:
                continue
            r = int(cells[es, 1])
            td = self.tokens[es]
            toks = [(td.terms[k], bool((r >> int(k)) & 1)) for k in td.order() if (p >> int(k)) & 1]
            out.append((self.elements.terms[es], toks))
        return out

    def decode_value_bits(self, words: np.ndarray) -> list:
        """value/1 bitmap -> element terms in term order."""
        out = []
        for es in self.elements.order():
            if (int(words[es >> 6]) >> int(es & 63)) & 1:
                out.append(self.elements.terms[es])
        return out

    # ------------------------------------------------------------------ wire codec
    def etf_arrays(self, E: int, tokens: bool = True):
        """The laspj_etf_dict_create arrays for E element slots: every registered term's
        external image (lasp_amd.etf.encode, once per term), element slots in term
        order (unregistered slots last) and, with `tokens`, per-element token images and
        token slots in term order."""
        from . import etf
        if self.size > E:
            raise CapacityError(f"{self.size} elements do not fit {E} slots")
        eoff = np.zeros((E + 1,), dtype=np.uint32)
        eparts = []
        for es, term in enumerate(self.elements.terms):
            img = etf.encode(term)
            eparts.append(img)
            eoff[es + 1] = len(img)
        eoff = np.cumsum(eoff, dtype=np.uint64).astype(np.uint32)
        order = np.concatenate([self.elements.order(),
                                np.arange(self.size, E, dtype=np.int64)]).astype(np.uint32)
        if not tokens:
            return b"".join(eparts), eoff, order, None, None, None
        tlen = np.zeros((64 * E + 1,), dtype=np.uint64)
        tparts = []
        tord = np.full((E, 64), 0xFF, dtype=np.uint8)
        for es, td in enumerate(self.tokens[:self.size]):
            # narrow cells hold token slots 0..63 (a wide domain's later slots are not
            # on this wire codec's cells)
            for k, term in enumerate(td.terms[:64]):
                img = etf.encode(term)
                tparts.append((64 * es + k, img))
                tlen[64 * es + k + 1] = len(img)
            o = td.order()
            o = o[o < 64]
            tord[es, :len(o)] = o
        toff = np.cumsum(tlen).astype(np.uint32)
        tparts.sort(key=lambda x: x[0])
        return (b"".join(eparts), eoff, order, b"".join(img for _k, img in tparts), toff,
                tord.reshape(-1))

    # ------------------------------------------------------------------ G-Set
    def encode_gset(self, states: Sequence, E: int) -> np.ndarray:
        for s in states:
            for elem in s:
                self.element_slot(elem)
        if self.size > E:
            raise CapacityError(f"{self.size} elements do not fit {E} slots")
        W = (E + 63) // 64
        out = np.zeros((len(states), W), dtype=np.uint64)
        for i, s in enumerate(states):
            _check_canonical_gset(s)
            for elem in s:
                es = self.element_slot(elem, create=False)
                out[i, es >> 6] |= np.uint64(1) << np.uint64(es & 63)
        return out

    def decode_gset(self, words: np.ndarray) -> list:
        return self.decode_value_bits(words)

    def keep_bits(self, pred, E: int) -> np.ndarray:
        """Evaluate a filter predicate once per element slot (lasp_core.erl:697)."""
        W = (E + 63) // 64
        out = np.zeros((W,), dtype=np.uint64)
        for es, elem in enumerate(self.elements.terms):
            if pred(elem) is True:
                out[es >> 6] |= np.uint64(1) << np.uint64(es & 63)
        return out


class _Journal:
    """O(1) to enter: the element count and the position in tok_log (every new token slot
    logs its element slot), from which a rollback knows what each token dictionary
    gained."""

    def __init__(self, dom: Domain):
        self.dom = dom

    def __enter__(self):
        d = self.dom
        self.ne = len(d.elements.terms)
        self.nlog = len(d.tok_log)
        return self

    def __exit__(self, et, ev, tb):
        if et is None:
            return False
        d = self.dom
        gained: Dict[int, int] = {}
        for es in d.tok_log[self.nlog:]:
            gained[es] = gained.get(es, 0) + 1
        for es, k in gained.items():
            if es < self.ne:
                td = d.tokens[es]
                td.truncate(len(td.terms) - k)
        del d.tokens[self.ne:]
        d.elements.truncate(self.ne)
        del d.tok_log[self.nlog:]
        return False


def _check_canonical_orset(s) -> None:
    prev = None
    for item in s:
        if not (isinstance(item, tuple) and len(item) == 2):
            raise NonCanonical(f"orddict entry {item!r} is not a 2-tuple")
        elem, toks = item
        if prev is not None and term_cmp(prev, elem) >= 0:
            raise NonCanonical("orddict keys are not strictly ascending")
        prev = elem
        if not isinstance(toks, list) or not toks:
            raise NonCanonical(f"element {elem!r} has an empty or non-list token orddict")
        tprev = None
        for t in toks:
            if not (isinstance(t, tuple) and len(t) == 2):
                raise NonCanonical("token orddict entry is not a 2-tuple")
            if tprev is not None and term_cmp(tprev, t[0]) >= 0:
                raise NonCanonical("token keys are not strictly ascending")
            tprev = t[0]


def _check_canonical_gset(s: Iterable) -> None:
    prev = None
    for e in s:
        if prev is not None and term_cmp(prev, e) >= 0:
            raise NonCanonical("ordset is not strictly ascending")
        prev = e


# ---------------------------------------------------------------------- combinator outputs

def decode_concat(dom: Domain, cells: np.ndarray) -> list:
    """CONCAT cells (E, 4) {pL, rL, pR, rR} -> the intersection body's list
    [{X, Cx ++ Cy}] in L's (term) order (lasp_core.erl:559-583, lasp_lattice.erl:311-312)."""
    out = []
    for es in dom.elements.order():
        if es >= cells.shape[0]:
            continue
        pl, rl, pr, rr = (int(v) for v in cells[es])
        if not pl:
            continue
        td = dom.tokens[es]
        cx = [(td.terms[k], bool((rl >> int(k)) & 1)) for k in td.order() if (pl >> int(k)) & 1]
        cy = [(td.terms[k], bool((rr >> int(k)) & 1)) for k in td.order() if (pr >> int(k)) & 1]
        out.append((dom.elements.terms[es], cx + cy))
    return out


def decode_product(dl: Domain, dr: Domain, cells: np.ndarray) -> list:
    """PRODUCT cells (EL, ER) uint32, or PRODUCT_WIDE cells (EL, ER, 4) uint64 -> the
    product body's list, X-major, each with orset_causal_product's fully reversed token
    order (lasp_lattice.erl:303-308)."""
    out = []
    wide = cells.ndim == 3
    xs = [int(x) for x in dl.elements.order() if x < cells.shape[0]]
    ys = [int(y) for y in dr.elements.order() if y < cells.shape[1]]
    for x in xs:
        row = cells[x]
        for y in ys:
            if wide:
                px, rx, py, ry = (int(v) for v in row[y])
                if not (px and py):
                    continue
            else:
                c = int(row[y])
                if not c:
                    continue
                px, rx, py, ry = c & 0xFF, (c >> 8) & 0xFF, (c >> 16) & 0xFF, (c >> 24) & 0xFF
            tdx, tdy = dl.tokens[x], dr.tokens[y]
            tx = [(tdx.terms[k], bool((rx >> int(k)) & 1)) for k in tdx.order() if (px >> int(k)) & 1]
            ty = [(tdy.terms[k], bool((ry >> int(k)) & 1)) for k in tdy.order() if (py >> int(k)) & 1]
            toks = [([a, b], da or db) for a, da in reversed(tx) for b, db in reversed(ty)]
            out.append(((dl.elements.terms[x], dr.elements.terms[y]), toks))
    return out


def decode_product_diag(dom: Domain, cells: np.ndarray) -> list:
    """laspj_orset_product_diag cells (E, 1) uint32 over one dictionary -> the list
    filter(fun({X, Y}) -> X =:= Y) leaves of the product body: {{X, X}, causal product}
    in X order (the product's X-major order restricted to its diagonal)."""
    out = []
    for x in dom.elements.order():
        x = int(x)
        if x >= cells.shape[0]:
            continue
        c = int(cells[x, 0])
        if not c:
            continue
        px, rx, py, ry = c & 0xFF, (c >> 8) & 0xFF, (c >> 16) & 0xFF, (c >> 24) & 0xFF
        td = dom.tokens[x]
        tx = [(td.terms[k], bool((rx >> int(k)) & 1)) for k in td.order() if (px >> int(k)) & 1]
        ty = [(td.terms[k], bool((ry >> int(k)) & 1)) for k in td.order() if (py >> int(k)) & 1]
        toks = [([a, b], da or db) for a, da in reversed(tx) for b, db in reversed(ty)]
        xt = dom.elements.terms[x]
        out.append(((xt, xt), toks))
    return out


def decode_gset_product(dl: Domain, dr: Domain, rows: np.ndarray) -> list:
    """G-Set product rows (EL, ceil(ER/64)) -> [{X, Y}] X-major (lasp_core.erl:518-520)."""
    out = []
    ys = [int(y) for y in dr.elements.order()]
    for x in dl.elements.order():
        x = int(x)
        if x >= rows.shape[0]:
            continue
        for y in ys:
            if (int(rows[x, y >> 6]) >> (y & 63)) & 1:
                out.append((dl.elements.terms[x], dr.elements.terms[y]))
    return out


class SeqOutput:
    """Output of the map / fold bodies (lasp_core.erl:641-667, 460-486): a list whose
    slot s holds key keys[s] with the causality of input slot src[s].  Slots are laid
    out in the input's list order, so decoding in slot order reproduces the reference's
    list exactly — unsorted or duplicated keys included."""

    def __init__(self, dom: Domain, keys: list, src: list):
        self.dom, self.keys, self.src = dom, keys, src

    # F runs once per dictionary element, not per replica.  A dictionary element that
    # F cannot take (F raises) keeps an empty slot: it is absent from every input that
    # reaches this body, or the reference's body would have crashed on it too.

    @classmethod
    def map(cls, dom: Domain, fun) -> "SeqOutput":
        keys, src = [], []
        for s in dom.elements.order():
            try:
                keys.append(fun(dom.elements.terms[int(s)]))
                src.append(int(s))
            except Exception:
                keys.append(None)
                src.append(0xFFFFFFFF)
        return cls(dom, keys, src)

    @classmethod
    def fold(cls, dom: Domain, fun) -> "SeqOutput":
        keys, src = [], []
        for s in dom.elements.order():
            try:
                vals = list(fun(dom.elements.terms[int(s)]))
            except Exception:
                continue
            for v in vals:
                keys.append(v)
                src.append(int(s))
        return cls(dom, keys, src)

    @property
    def size(self) -> int:
        return len(self.keys)

    def index(self) -> np.ndarray:
        return np.asarray(self.src if self.src else [0xFFFFFFFF], dtype=np.uint32)

    def decode_orset(self, cells: np.ndarray) -> list:
        out = []
        for o, (key, s) in enumerate(zip(self.keys, self.src)):
            p, r = int(cells[o, 0]), int(cells[o, 1])
            if not p or s == 0xFFFFFFFF:
                continue
            td = self.dom.tokens[s]
            out.append((key, [(td.terms[k], bool((r >> int(k)) & 1))
                              for k in td.order() if (p >> int(k)) & 1]))
        return out

    def decode_bits(self, words: np.ndarray) -> list:
        return [key for o, key in enumerate(self.keys) if (int(words[o >> 6]) >> (o & 63)) & 1]
