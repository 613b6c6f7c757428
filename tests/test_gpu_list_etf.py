"""The combinator bodies and bind/3 on list values from term_to_binary images
(include/laspj.h "list bodies from images", lasp_amd/csrc/laspj_list_etf.cpp) against the
oracle's bodies (oracle/core.py, restating lasp_core.erl:460-712) and bind
(lasp_core.erl:291-312 with orddict:merge / ordsets:union run as written), on the parity
traps of SURVEY.md Appendix B: union keeping the left tokens, the G-Set `L ++ R` with
overlap, intersection's `Cx ++ Cy` duplicates, product's descending token pairs, collapsing
maps and folds with duplicate keys, filter keeping tombstones, re-binding unsorted lists
(keyfind first match: a merge that is not an inflation), and the values that go back to the
reference's own body (FALLBACK).  The same cases run from plain C on four threads
(tests/c/laspj_nif_threads.c, with G-Set image calls and resident variables)."""

import random

import pytest

from oracle import core as ocore
from oracle import etf as oetf
from oracle import gset as ogset
from oracle import lattice as olat
from oracle import orset as oorset
from oracle import otp
from oracle.terms import Atom, exact_eq

OK, FALLBACK = 0, 1
BODY = {"union": 0, "intersection": 1, "product": 2, "map": 3, "filter": 4, "fold": 5,
        "value": 6, "bind": 7}


def _tb(t) -> bytes:
    return oetf.term_to_binary(t)


def _tok(rng):
    return bytes(rng.getrandbits(8) for _ in range(20))


def _orddict(rng, keys, tmax=3, pflag=0.3):
    return [(k, sorted([(_tok(rng), rng.random() < pflag) for _ in range(rng.randint(1, tmax))]))
            for k in sorted(keys)]


def _args(kind, value):
    """The distinct values the body passes its fun, first appearance first."""
    out = []
    for e in value:
        a = e[0] if isinstance(e, tuple) and len(e) == 2 else e
        if not any(exact_eq(a, x) for x in out):
            out.append(a)
    return out


def _bind_oracle(kind, v0, v):
    t = "lasp_gset" if kind == "gset" else "lasp_orset"
    if exact_eq(v0, v):
        return 0, None
    m = (ogset if kind == "gset" else oorset).merge(v0, v)
    return (1, m) if olat.is_inflation(t, v0, m) else (2, None)


def _fun_case(kind, body, value, fun):
    """(op, verdict, result, a, b, expected) for map / filter / fold: b = the image of the
    fun's results over the distinct arguments."""
    t = "lasp_gset" if kind == "gset" else "lasp_orset"
    res = [fun(a) for a in _args(kind, value)]
    want = getattr(ocore, body + "_body")(t, fun, value)
    return ((120 if kind == "gset" else 20) + BODY[body], OK, 0, _tb(value), _tb(res), _tb(want))


def list_cases(seed=1):
    rng = random.Random(seed)
    O, G = 20, 120
    A = _orddict(rng, rng.sample(range(40), 18))
    B = _orddict(rng, rng.sample(range(40), 18))
    tomb = [(k, [(t, True) for t, _f in ts]) for k, ts in A[:5]] + A[5:]
    cases = []
    add = lambda op, a, b, want: cases.append((op, OK, 0, _tb(a), _tb(b), _tb(want)))  # noqa: E731
    # union: keep-left tokens (Appendix B1); unsorted inputs run through the two-finger walk
    isect_ab = ocore.intersection_body("lasp_orset", A, B)
    mapped = ocore.map_body("lasp_orset", lambda x: 40 - x, A)          # descending keys
    for l, r in [(A, B), (B, A), (mapped, B), (B, mapped), (isect_ab, A), ([], A), (A, [])]:
        add(O + 0, l, r, ocore.union_body("lasp_orset", l, r))
    # G-Set union = L ++ R (Appendix B2: overlap kept, unsorted)
    for l, r in [([1, 2, 3], [2, 3, 4]), ([Atom("b"), 5], [Atom("a"), 5]), ([], [7]),
                 ([(1, 2)], [300, b"x"])]:
        add(G + 0, l, r, ocore.union_body("lasp_gset", l, r))
    # intersection: Cx ++ Cy, self-intersection duplicates (B4), keyfind first match on a
    # list with repeated keys
    rep = A[:4] + [(A[1][0], [(_tok(rng), False)])] + A[4:]
    for l, r in [(A, B), (A, A), (isect_ab, A), (rep, rep), (mapped, A), (A, [])]:
        add(O + 1, l, r, ocore.intersection_body("lasp_orset", l, r))
    for l, r in [([1, 2, 3, 2], [3, 2, 9]), ([Atom("x"), b"y"], [b"y"])]:
        add(G + 1, l, r, ocore.intersection_body("lasp_gset", l, r))
    # product: X-major pairs, token pairs fully descending (B3)
    for l, r in [(A[:6], B[:5]), (B[:3], A[:7]), ([], A[:3])]:
        add(O + 2, l, r, ocore.product_body("lasp_orset", l, r))
    add(G + 2, [1, 2, 3], [Atom("a"), 3], ocore.product_body("lasp_gset", [1, 2, 3], [Atom("a"), 3]))
    # map / filter / fold (the fun evaluated over the distinct arguments)
    cases.append(_fun_case("orset", "map", A, lambda x: x // 3))                 # collapsing
    cases.append(_fun_case("orset", "map", rep, lambda x: (Atom("k"), x % 4)))
    cases.append(_fun_case("orset", "filter", tomb, lambda x: x % 2 == 0))       # B6
    cases.append(_fun_case("orset", "filter", isect_ab, lambda x: Atom("maybe") if x % 3 else True))
    cases.append(_fun_case("orset", "fold", A, lambda x: [x, x, x]))            # B5
    cases.append(_fun_case("orset", "fold", mapped, lambda x: [x % 5, x + 100] if x % 2 else []))
    gl = [5, 1, 9, 1, (Atom("a"), 3), (Atom("b"), [1])]
    cases.append(_fun_case("gset", "map", gl, lambda x: x * 2 if isinstance(x, int) else [x]))
    cases.append(_fun_case("gset", "filter", gl, lambda x: x != 1))
    cases.append(_fun_case("gset", "fold", gl, lambda x: [x, x] if isinstance(x, int) else [0]))
    # value/1 of list values: keys with a false token, list order
    for v in (isect_ab, tomb, rep, mapped):
        add(O + 6, v, [], oorset.value(v))
    add(G + 6, [3, 1, 3], [], [3, 1, 3])
    # bind/3 on lists: no-op, writes, and a merge that is not an inflation (keyfind pairs
    # a repeated key's second entry with the first one)
    dup = [(1, [(b"a" * 20, False)]), (1, [(b"b" * 20, False)])]
    for kind, v0, v in [("orset", isect_ab, isect_ab), ("orset", isect_ab, A),
                        ("orset", mapped, B), ("orset", dup, [(1, [(b"c" * 20, False)])]),
                        ("orset", [], rep), ("gset", [3, 1, 2], [2, 5]),
                        ("gset", [1, 2, 3, 2, 3, 4], [1, 2, 3, 2, 3, 4]),
                        ("gset", [5, 1], [1, 5])]:
        st, m = _bind_oracle(kind, v0, v)
        op = (G if kind == "gset" else O) + BODY["bind"]
        cases.append((op, OK, st, _tb(v0), _tb(v), _tb(m) if m is not None else b""))
    return cases


def fallback_list_cases(seed=2):
    rng = random.Random(seed)
    good = [(1, [(_tok(rng), False)])]
    t = sorted(_tok(rng) for _ in range(70))
    bad = {
        "improper": _tb(good)[:-1] + bytes([97, 3]),
        "entry not a pair": _tb([(1, [(t[0], False)], 3)]),
        "flag not a boolean": _tb([(1, [(t[0], Atom("maybe"))])]),
        "65 tokens on a key": _tb([(1, [(x, False) for x in t[:65]])]),
        "1 and 1.0": _tb([(1, [(t[1], False)]), (1.0, [(t[2], False)])]),
        "not a list": _tb(Atom("a")),
    }
    out = []
    for name, img in bad.items():
        out.append((20, FALLBACK, 0, _tb(good), img, b""))
        out.append((21, FALLBACK, 0, img, _tb(good), b""))
    # G-Set intersection / product over 2-tuple elements: the OR-Set branch with a non-list
    # causality is the reference's to run
    out.append((121, FALLBACK, 0, _tb([(Atom("a"), 1)]), _tb([(Atom("a"), 2)]), b""))
    out.append((122, FALLBACK, 0, _tb([1]), _tb([(1, 2)]), b""))
    return out


def _run(ctx, case):
    op, verdict, result, a, b, exp = case
    kind = "gset" if op >= 120 else "orset"
    k = op - (120 if op >= 120 else 20)
    name = {v: n for n, v in BODY.items()}[k]
    if name == "bind":
        v, st, img = ctx.list_etf_bind(kind, a, b)
        return v, (st, img)
    return ctx.list_etf(name, kind, a, b)


def _check(case, got):
    op, verdict, result, a, b, exp = case
    v, ans = got
    assert v == verdict, (op, v, verdict)
    if v != OK:
        return
    if (op - 20) % 100 == BODY["bind"]:
        st, img = ans
        assert st == result, (op, st, result)
        if st == 1:
            assert img == exp, op
    else:
        assert ans == exp, (op, oetf.binary_to_term(ans) if ans else ans,
                            oetf.binary_to_term(exp))


@pytest.mark.gpu
def test_list_bodies_from_images_match_oracle():
    from lasp_amd import engine
    ctx = engine.Context(0)
    try:
        for case in list_cases(1) + list_cases(7) + fallback_list_cases():
            _check(case, _run(ctx, case))
    finally:
        ctx.close()


@pytest.mark.gpu
def test_list_args_are_the_distinct_fun_arguments():
    """laspj_list_etf_args: what the NIF maps the fun over — keys (OR-Set), elements or a
    2-tuple element's first component (G-Set), first appearance first."""
    from lasp_amd import engine
    ctx = engine.Context(0)
    try:
        rng = random.Random(3)
        A = _orddict(rng, range(12))
        rep = A + A[:3]
        for kind, v in [("orset", A), ("orset", rep), ("orset", []),
                        ("gset", [5, 1, 5, (Atom("a"), 2), (Atom("a"), 3), 7])]:
            assert ctx.list_etf("args", kind, _tb(v)) == (OK, _tb(_args(kind, v)))
        # a result list of the wrong length is an argument error
        from lasp_amd import _lib
        with pytest.raises(_lib.LaspjError):
            ctx.list_etf("map", "orset", _tb(A), _tb([1, 2]))
    finally:
        ctx.close()


def _var_cases(seed=4):
    rng = random.Random(seed)
    A = _orddict(rng, rng.sample(range(30), 12))
    B = _orddict(rng, rng.sample(range(30), 12))
    out = []
    for a, b in [(A, B), (A, A), ([], A), (B, [])]:
        st, m = _bind_oracle("orset", a, b)
        out.append((10, OK, st, _tb(a), _tb(b), _tb(m if m is not None else a)))
    for a, b in [([1, 5], [2, 5]), ([3], [3]), ([], [Atom("z")])]:
        st, m = _bind_oracle("gset", a, b)
        out.append((11, OK, st, _tb(a), _tb(b), _tb(m if m is not None else a)))
    return out


def _gset_image_cases(seed=5):
    rng = random.Random(seed)
    pool = list(range(0, 90, 3)) + [Atom(f"a{k}") for k in range(6)] + [b"x", b"yy", (1, 2)]
    out = []
    for k in range(10):
        a = otp.lists_usort(rng.sample(pool, 12))
        b = otp.lists_usort(rng.sample(pool, 12))
        out.append((5, OK, 0, _tb(a), _tb(b), _tb(ogset.merge(a, b))))
        out.append((6, OK, 0, _tb(a), b"", _tb(a)))
        out.append((7, OK, int(ogset.equal(a, a if k % 2 else b)), _tb(a),
                    _tb(a if k % 2 else b), b""))
        m = ogset.merge(a, b)
        out.append((8, OK, int(olat.is_inflation("lasp_gset", a, m)), _tb(a), _tb(m), b""))
        out.append((9, OK, int(olat.is_strict_inflation("lasp_gset", a, a if k % 3 == 0 else m)),
                    _tb(a), _tb(a if k % 3 == 0 else m), b""))
    out.append((5, FALLBACK, 0, _tb([1]), _tb([3, 2]), b""))
    return out


@pytest.mark.gpu
def test_list_gset_var_cases_from_plain_c(tmp_path):
    """tests/c/laspj_nif_threads.c on 4 threads x 4 contexts: list bodies and binds from
    images, G-Set image calls and resident variables, through laspj.h alone."""
    import subprocess
    from test_gpu_nif import _build_threads_exe, write_cases
    exe = _build_threads_exe(tmp_path)
    p = tmp_path / "cases.bin"
    write_cases(p, list_cases(11) + fallback_list_cases(12) + _var_cases() + _gset_image_cases())
    res = subprocess.run([exe, str(p), "4"], capture_output=True, text=True, timeout=240)
    assert res.returncode == 0, res.stdout + res.stderr
    assert "laspj NIF threads OK" in res.stdout


def test_list_cases_are_the_oracles_answers():
    """(CPU) the case generator's expected images decode to the oracle's terms."""
    cases = list_cases(1)
    assert len(cases) > 40
    for op, verdict, result, a, b, exp in cases:
        assert verdict == OK
        oetf.binary_to_term(a)
        if exp:
            oetf.binary_to_term(exp)


@pytest.mark.gpu
def test_list_images_fuzz_answer_or_fall_back():
    """Mutated images (truncated, a byte flipped, junk appended, a tag byte replaced) into
    the list bodies and bind: every call answers FALLBACK, raises an error status, or
    answers OK with the oracle body's answer on the terms the mutated images decode to —
    never a crash (the NIF runs inside the BEAM) and never a wrong OK."""
    from lasp_amd import _lib, engine
    ctx = engine.Context(0)
    rng = random.Random(99)
    try:
        A = _orddict(rng, rng.sample(range(40), 10))
        B = _orddict(rng, rng.sample(range(40), 10))
        bases = [("orset", "union", A, B), ("orset", "intersection", A, B),
                 ("orset", "product", A[:4], B[:4]), ("orset", "bind", A, B),
                 ("gset", "union", [1, 5, 9, Atom("x")], [5, 2, b"q"]),
                 ("gset", "bind", [1, 5, 9], [2, 5])]

        def mutate(img):
            b = bytearray(img)
            k = rng.randrange(4)
            if k == 0 and len(b) > 2:
                return bytes(b[:rng.randrange(1, len(b))])
            if k == 1:
                i = rng.randrange(len(b))
                b[i] ^= 1 << rng.randrange(8)
                return bytes(b)
            if k == 2:
                return bytes(b) + bytes(rng.getrandbits(8) for _ in range(rng.randint(1, 6)))
            i = rng.randrange(1, len(b))
            b[i] = rng.choice([97, 98, 100, 104, 106, 107, 108, 109, 110, 115, 118, 119])
            return bytes(b)

        answered = 0
        for n in range(3000):
            kind, body, a, b = bases[n % len(bases)]
            ia, ib = _tb(a), _tb(b)
            if n % 2:
                ia = mutate(ia)
            else:
                ib = mutate(ib)
            try:
                if body == "bind":
                    verd, st, img = ctx.list_etf_bind(kind, ia, ib)
                else:
                    verd, img = ctx.list_etf(body, kind, ia, ib)
            except _lib.LaspjError:
                continue
            assert verd in (OK, FALLBACK)
            if verd != OK:
                continue
            # an OK answer: the mutated images are terms the body takes, and the answer is
            # the oracle's
            ta, tb_ = oetf.binary_to_term(ia), oetf.binary_to_term(ib)
            t = "lasp_gset" if kind == "gset" else "lasp_orset"
            if body == "bind":
                want_st, m = _bind_oracle(kind, ta, tb_)
                assert st == want_st, (ta, tb_)
                if st == 1:
                    assert exact_eq(oetf.binary_to_term(img), m)
            else:
                want = getattr(ocore, body + "_body")(t, ta, tb_)
                assert exact_eq(oetf.binary_to_term(img), want), (body, ta, tb_)
            answered += 1
        assert answered > 0
    finally:
        ctx.close()
