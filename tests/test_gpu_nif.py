"""The NIF-level entry points (include/laspj.h "NIF entry points", lasp_amd/csrc/laspj_nif.hip):
term_to_binary images in, the reference's answer out — merge/2, value/1, equal/2 and
is_(strict_)inflation — against the oracle (oracle/orset.py, oracle/lattice.py, the ETF
restatement oracle/etf.py), including the verdicts that hand an operand back to the
reference's own Erlang clause, the registration of unseen terms, dictionary resets, the
host-encoded path for token images of mixed lengths, and several schedulers (threads) on
their own contexts at once — from Python (ctypes) and from plain C (tests/c/laspj_nif_threads.c).

Reference: lasp_orset.erl:67-73 (value/1), :128-134 (merge/2), :136-138 (equal/2);
lasp_lattice.erl:153-161, 235-253 (inflation); lasp_core.erl:298-311 (bind/3 calls merge).
"""

import functools
import os
import random
import struct
import subprocess
import threading

import pytest

from oracle import etf as oetf
from oracle import lattice as olat
from oracle import orset as oorset
from oracle.terms import Atom, compare

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
OK, FALLBACK = 0, 1
MERGE, VALUE, EQUAL, INFL, SINFL = 0, 1, 2, 3, 4

_key = functools.cmp_to_key(compare)


def _tb(t) -> bytes:
    return oetf.term_to_binary(t)


def _tokens(rng, n, size=20):
    return [bytes(rng.getrandbits(8) for _ in range(size)) for _ in range(n)]


def _orset(rng, elems, pool, p=0.7, pflag=0.3, tmax=None):
    s = []
    for e in elems:
        if rng.random() < p:
            ts = pool[e]
            k = rng.randint(1, min(len(ts), tmax or len(ts)))
            toks = sorted(rng.sample(ts, k), key=_key)
            s.append((e, [(t, rng.random() < pflag) for t in toks]))
    return s


def _universe(rng, n_elems, toks_per=6, size=20):
    elems = list(range(n_elems // 2)) + [Atom(f"e{k}") for k in range(n_elems // 4)] + \
        [f"b{k}".encode() for k in range(n_elems - n_elems // 2 - n_elems // 4)]
    elems = sorted(elems, key=_key)
    pool = {e: _tokens(rng, toks_per, size) for e in elems}
    return elems, pool


def valid_cases(seed=1, n=24, n_elems=40):
    """(op, verdict, result, a, b, expected image) on canonical orddicts."""
    rng = random.Random(seed)
    elems, pool = _universe(rng, n_elems)
    out = []
    for k in range(n):
        a = _orset(rng, elems, pool)
        b = _orset(rng, elems, pool)
        m = oorset.merge(a, b)
        out.append((MERGE, OK, 0, _tb(a), _tb(b), _tb(m)))
        out.append((VALUE, OK, 0, _tb(a), b"", _tb(oorset.value(a))))
        same = a if k % 3 == 0 else b
        out.append((EQUAL, OK, int(oorset.equal(a, same)), _tb(a), _tb(same), b""))
        cur = m if k % 2 == 0 else b
        out.append((INFL, OK, int(olat.is_inflation("lasp_orset", a, cur)), _tb(a), _tb(cur), b""))
        cur = a if k % 4 == 0 else cur
        out.append((SINFL, OK, int(olat.is_strict_inflation("lasp_orset", a, cur)), _tb(a),
                    _tb(cur), b""))
    # empty operands
    out.append((MERGE, OK, 0, _tb([]), _tb([]), _tb([])))
    a = _orset(rng, elems, pool)
    out.append((MERGE, OK, 0, _tb([]), _tb(a), _tb(oorset.merge([], a))))
    out.append((VALUE, OK, 0, _tb([]), b"", _tb([])))
    out.append((SINFL, OK, 1 if a else 0, _tb([]), _tb(a), b""))
    return out


def _pid_like_payload(tok: bytes) -> bytes:
    """An orddict whose element is a map (#{}): a term kind no dictionary holds."""
    el = bytes([116, 0, 0, 0, 0])
    rec = bytes([104, 2, 109]) + struct.pack(">I", len(tok)) + tok + _tb(False)[1:]
    return bytes([131, 108, 0, 0, 0, 1, 104, 2]) + el + bytes([108, 0, 0, 0, 1]) + rec + \
        bytes([106, 106])


def fallback_cases(seed=2):
    """Operands the columnar path does not take: verdict FALLBACK (the NIF runs the
    reference's Erlang clause, which answers or crashes as the reference does) — after
    the answers of a wide element (65 tokens), so the wide decoder meets them too."""
    rng = random.Random(seed)
    t = _tokens(rng, 70)
    good = [(1, [(t[0], False)]), (2, [(t[1], True)])]
    bad = {
        "keys descend": [(2, [(t[0], False)]), (1, [(t[1], False)])],
        "key twice": [(1, [(t[0], False)]), (1, [(t[1], False)])],
        "tokens descend": [(1, sorted([(t[2], False), (t[3], False)], reverse=True))],
        "65 tokens of two lengths": [(1, sorted([(x, False) for x in t[:64]] +
                                                [(t[65] + b"x", False)], key=_key))],
        "no tokens": [(1, [])],
        "not a list": (1, 2),
        "flag not a boolean": [(1, [(t[4], Atom("maybe"))])],
        "entry not a pair": [(1, [(t[5], False)], 3)],
    }
    out = []
    for name, v in bad.items():
        out.append((MERGE, FALLBACK, 0, _tb(good), _tb(v), b""))
        out.append((MERGE, FALLBACK, 0, _tb(v), _tb(good), b""))
        out.append((VALUE, FALLBACK, 0, _tb(v), b"", b""))
        out.append((EQUAL, FALLBACK, 0, _tb(v), _tb(good), b""))
        out.append((INFL, FALLBACK, 0, _tb(good), _tb(v), b""))
    p = _pid_like_payload(t[6])
    out.append((MERGE, FALLBACK, 0, _tb(good), p, b""))
    out.append((VALUE, FALLBACK, 0, p, b"", b""))
    # an element of 65 tokens (the reference mints one per add and never collects them,
    # lasp_orset.erl:222-241): the namespace goes wide (k {p, r} pairs per cell) and
    # answers; the operands after it still fall back as above
    wide = [(1, [(x, k % 3 == 0) for k, x in enumerate(sorted(t[:65]))])]
    out.insert(0, (MERGE, OK, 0, _tb(good), _tb(wide), _tb(oorset.merge(good, wide))))
    out.insert(1, (MERGE, OK, 0, _tb(wide), _tb(good), _tb(oorset.merge(wide, good))))
    out.insert(2, (VALUE, OK, 0, _tb(wide), b"", _tb(oorset.value(wide))))
    out.insert(3, (EQUAL, OK, 0, _tb(wide), _tb(good), b""))
    out.insert(4, (INFL, OK, int(olat.is_inflation("lasp_orset", good, wide)), _tb(good),
                   _tb(wide), b""))
    out.insert(5, (SINFL, OK, int(olat.is_strict_inflation("lasp_orset", wide, wide)),
                   _tb(wide), _tb(wide), b""))
    return out


def write_cases(path, cases):
    with open(path, "wb") as f:
        f.write(struct.pack("<I", len(cases)))
        for op, verdict, result, a, b, exp in cases:
            f.write(struct.pack("<Iii", op, verdict, result))
            for blob in (a, b, exp):
                f.write(struct.pack("<Q", len(blob)))
                f.write(blob)


def _build_threads_exe(tmp_path):
    import shutil
    cc = shutil.which("gcc") or shutil.which("cc")
    if cc is None:
        pytest.skip("no C compiler")
    exe = str(tmp_path / "laspj_nif_threads")
    libdir = os.path.join(ROOT, "lasp_amd")
    cmd = [cc, "-std=c11", "-O2", "-Wall", "-Werror", "-pthread", "-I",
           os.path.join(ROOT, "include"), os.path.join(ROOT, "tests", "c", "laspj_nif_threads.c"),
           "-L", libdir, "-llaspj", f"-Wl,-rpath,{libdir}", "-o", exe]
    res = subprocess.run(cmd, capture_output=True, text=True)
    assert res.returncode == 0, res.stderr
    return exe


# ------------------------------------------------------------------ CPU side

def test_nif_threads_client_compiles(tmp_path):
    _build_threads_exe(tmp_path)


def test_nif_cases_are_the_oracles_answers(tmp_path):
    """The case file round-trips, and its expected images decode to the oracle's terms
    (so the GPU tests compare against the reference's algorithm, not a copy of the
    device's output)."""
    cases = valid_cases(n=6) + fallback_cases()
    p = tmp_path / "cases.bin"
    write_cases(p, cases)
    raw = p.read_bytes()
    assert struct.unpack_from("<I", raw)[0] == len(cases)
    for op, verdict, result, a, b, exp in cases:
        if op == MERGE and verdict == OK:
            assert oetf.binary_to_term(exp) == oorset.merge(oetf.binary_to_term(a),
                                                             oetf.binary_to_term(b))


# ------------------------------------------------------------------ GPU side

def _ctx():
    from lasp_amd import engine
    return engine.Context(0)


def _run_case(ctx, case):
    op, verdict, result, a, b, exp = case
    if op == MERGE:
        v, img = ctx.nif_merge(a, b)
        return v, img
    if op == VALUE:
        return ctx.nif_value(a)
    if op == EQUAL:
        return ctx.nif_equal(a, b)
    return ctx.nif_inflation(a, b, strict=(op == SINFL))


def _check(case, got):
    op, verdict, result, a, b, exp = case
    v, ans = got
    assert v == verdict, (op, v, verdict)
    if verdict != OK:
        assert ans is None
    elif op in (MERGE, VALUE):
        assert ans == exp, (op, len(ans), len(exp))
    else:
        assert ans == bool(result), (op, ans, result)


@pytest.mark.gpu
def test_nif_answers_match_oracle():
    ctx = _ctx()
    try:
        for case in valid_cases(seed=11, n=30) + fallback_cases(seed=12):
            _check(case, _run_case(ctx, case))
        st = ctx.nif_stats()
        assert st["fallbacks"] > 0 and st["registrations"] > 0
    finally:
        ctx.close()


@pytest.mark.gpu
def test_nif_unknown_terms_register_once_then_one_pass():
    """A fresh token makes the decoder answer UNKNOWN_TERM: the call registers and runs a
    second pass; the same operands again take one device pass and no registration."""
    ctx = _ctx()
    try:
        rng = random.Random(5)
        elems, pool = _universe(rng, 64)
        a, b = _orset(rng, elems, pool), _orset(rng, elems, pool)
        want = _tb(oorset.merge(a, b))
        assert ctx.nif_merge(_tb(a), _tb(b)) == (OK, want)
        s0 = ctx.nif_stats()
        for _ in range(3):
            assert ctx.nif_merge(_tb(a), _tb(b)) == (OK, want)
        s1 = ctx.nif_stats()
        assert s1["registrations"] == s0["registrations"]
        assert s1["device_passes"] - s0["device_passes"] == 3
        # an update mints a token (lasp_orset.erl:222-230, 261-262): one new term
        e = elems[3]
        b2 = oorset.merge(b, [(e, [(b"\x01" * 20, False)])])
        assert ctx.nif_merge(_tb(a), _tb(b2)) == (OK, _tb(oorset.merge(a, b2)))
        s2 = ctx.nif_stats()
        assert s2["registrations"] == s1["registrations"] + 1
        assert s2["device_passes"] == s1["device_passes"] + 2
    finally:
        ctx.close()


@pytest.mark.gpu
def test_nif_new_tokens_patch_the_device_images():
    """Replicas exchanging state after updates: every merge meets tokens the dictionary
    has not seen, on elements it holds.  Those registrations patch the device images in
    place (etf_dict_patch: token mask, term order, writer descriptors, record templates,
    bucket tables of the elements concerned) instead of rebuilding them; an element that
    outgrows its token headroom, or a new element, rebuilds.  Every answer is the
    oracle's, image for image, across 60 rounds in which the state keeps growing."""
    ctx = _ctx()
    try:
        rng = random.Random(77)
        elems = list(range(0, 900, 3))
        mk = lambda: bytes(rng.getrandbits(8) for _ in range(20))  # noqa: E731
        a = [(e, [(mk(), rng.random() < 0.3)]) for e in elems]
        b = [(e, [(mk(), rng.random() < 0.3)]) for e in elems if rng.random() < 0.8]
        cur = oorset.merge(a, b)
        assert ctx.nif_merge(_tb(a), _tb(b)) == (OK, _tb(cur))
        s0 = ctx.nif_stats()
        for rnd in range(60):
            # the other replica's update: new tokens on a few known elements (its own
            # earlier tokens kept), now and then a new element, a removal flag set
            other = dict((e, list(ts)) for e, ts in cur)
            for e in rng.sample(elems, rng.randint(1, 6)):
                other.setdefault(e, []).append((mk(), rng.random() < 0.2))
            if rnd % 17 == 16:
                other[901 + rnd] = [(mk(), False)]
            for e in rng.sample(list(other), 3):
                ts = other[e]
                j = rng.randrange(len(ts))
                ts[j] = (ts[j][0], True)
            o = sorted(((e, sorted(ts, key=lambda x: _key(x[0]))) for e, ts in other.items()),
                       key=lambda x: _key(x[0]))
            want = oorset.merge(cur, o)
            got = ctx.nif_merge(_tb(cur), _tb(o))
            assert got == (OK, _tb(want)), rnd
            cur = want
        s1 = ctx.nif_stats()
        assert s1["image_patches"] - s0["image_patches"] >= 30
        assert s1["image_rebuilds"] - s0["image_rebuilds"] < 30
        assert s1["fallbacks"] == s0["fallbacks"]
        # the chain checked beside the join gives a new token's UNKNOWN_TERM exactly (the
        # failing segment started where the serial decoder would be): no serial pass for
        # those; only a new element (its header resolves nowhere) may take one
        assert s1["chain_redo_passes"] - s0["chain_redo_passes"] <= 3
    finally:
        ctx.close()


@pytest.mark.gpu
def test_nif_false_element_headers_in_tokens_take_the_serial_pass():
    """Tokens that embed a real element header (106 104 2 97 e 108) plant false segment
    starts in 256-byte segments: the chain checked beside the join breaks, the call decodes
    again serially (chain_redo_passes) and answers the oracle's merge, image for image.
    Then a new token deep in a 10k-element operand: its segment's UNKNOWN_TERM is exact
    (no serial pass), the call registers it and answers the oracle's merge."""
    from lasp_amd import _lib
    ctx = _ctx()
    try:
        ctx.set_tuning(_lib.TUNE_ETF_SEG, 256)
        rng = random.Random(31)
        trap = lambda e, k: bytes([106, 104, 2, 97, e, 108]) + bytes([k]) * 14   # noqa: E731
        tok = lambda e, k: (trap((e + 7) % 200, k) if e % 5 == 0  # noqa: E731
                            else bytes([k, e % 256]) * 10)
        # >= 1024 element slots: the merge is the fused join the chain check rides on
        a = [(e, sorted([(tok(e, k), rng.random() < 0.3) for k in range(2)],
                        key=lambda x: _key(x[0]))) for e in range(1200)]
        b = [(e, sorted([(tok(e, k), rng.random() < 0.3) for k in range(1, 3)],
                        key=lambda x: _key(x[0]))) for e in range(0, 1200, 2)]
        want = _tb(oorset.merge(a, b))
        assert ctx.nif_merge(_tb(a), _tb(b)) == (OK, want)
        s0 = ctx.nif_stats()
        assert ctx.nif_merge(_tb(a), _tb(b)) == (OK, want)          # warm
        s1 = ctx.nif_stats()
        assert s1["chain_redo_passes"] > s0["chain_redo_passes"]
        assert s1["registrations"] == s0["registrations"]
        # value/1 of such an operand: its chain check rides on the answer's size pass, and
        # breaks the same way
        assert ctx.nif_value(_tb(a)) == (OK, _tb(oorset.value(a)))
        s1v = ctx.nif_stats()
        assert s1v["chain_redo_passes"] > s1["chain_redo_passes"]
        ctx.set_tuning(_lib.TUNE_ETF_SEG, 0)
        big = [(e, [(bytes([e % 251, e // 251]) * 10, False)]) for e in range(10_000)]
        other = [(e, list(ts)) for e, ts in big]
        assert ctx.nif_merge(_tb(big), _tb(other)) == (OK, _tb(big))
        s2 = ctx.nif_stats()
        other[7777] = (7777, sorted(other[7777][1] + [(b"\x05" * 20, True)],
                                    key=lambda x: _key(x[0])))
        assert ctx.nif_merge(_tb(big), _tb(other)) == (OK, _tb(oorset.merge(big, other)))
        s3 = ctx.nif_stats()
        assert s3["registrations"] == s2["registrations"] + 1
        assert s3["chain_redo_passes"] == s2["chain_redo_passes"]
    finally:
        ctx.close()


@pytest.mark.gpu
def test_nif_one_launch_merge_edges():
    """The single merge written in one launch (look-back over 256-element chunks) once the
    context's dictionary holds >= 1024 element slots: an empty answer ([] with [] -> the
    list header alone, 131 106), answers whose present elements sit in one chunk or at
    the ends, and an operand of one element — each the oracle's image."""
    ctx = _ctx()
    try:
        rng = random.Random(41)
        tok = lambda e, k: bytes([k, e % 251, e // 251]) + bytes(17)   # noqa: E731
        big = [(e, [(tok(e, 0), False)]) for e in range(1500)]
        assert ctx.nif_merge(_tb(big), _tb(big)) == (OK, _tb(big))
        cases = [([], []),
                 ([], big[:1]),
                 (big[700:760], big[730:800]),
                 (big[:3], big[-3:]),
                 ([(e, [(tok(e, 0), True)]) for e in range(0, 1500, 97)], big[::250])]
        for a, b in cases:
            assert ctx.nif_merge(_tb(a), _tb(b)) == (OK, _tb(oorset.merge(a, b))), (len(a), len(b))
        assert ctx.nif_stats()["registrations"] >= 1
    finally:
        ctx.close()


@pytest.mark.gpu
def test_nif_dictionary_reset_when_an_element_runs_out_of_token_slots():
    """Calls are self-contained, so a context whose dictionary has given an element all 64
    token slots starts a fresh dictionary for a call that needs more (and answers it)."""
    ctx = _ctx()
    try:
        rng = random.Random(6)
        for k in range(4):                      # 4 x 40 distinct tokens on element 1
            toks = sorted(_tokens(rng, 40))
            a = [(1, [(t, False) for t in toks[:20]])]
            b = [(1, [(t, bool(i % 2)) for i, t in enumerate(toks[20:])])]
            assert ctx.nif_merge(_tb(a), _tb(b)) == (OK, _tb(oorset.merge(a, b)))
        st = ctx.nif_stats()
        assert st["dict_resets"] >= 2 and st["fallbacks"] == 0
        assert st["dict_elements"] <= 2
    finally:
        ctx.close()


@pytest.mark.gpu
def test_nif_merge_many_mixed_verdicts():
    ctx = _ctx()
    try:
        rng = random.Random(7)
        elems, pool = _universe(rng, 48)
        pairs, want = [], []
        bad = [(2, [(b"x" * 20, False)]), (1, [(b"y" * 20, False)])]
        for k in range(40):
            a, b = _orset(rng, elems, pool), _orset(rng, elems, pool)
            if k % 7 == 3:
                pairs.append((_tb(a), _tb(bad)))
                want.append((FALLBACK, None))
            else:
                pairs.append((_tb(a), _tb(b)))
                want.append((OK, _tb(oorset.merge(a, b))))
        assert ctx.nif_merge_many(pairs) == want
        assert ctx.nif_merge_many(pairs) == want          # warm: no registration
    finally:
        ctx.close()


@pytest.mark.gpu
def test_nif_mixed_token_image_lengths_take_the_host_encoder():
    """Token images of several lengths: the device decoder needs one length, so the
    context's host dictionary encodes the cells and the device does the rest."""
    ctx = _ctx()
    try:
        rng = random.Random(8)
        elems = list(range(30))
        pool = {e: _tokens(rng, 3, 20) + _tokens(rng, 2, 33) + [e * 1000 + 7] for e in elems}
        for e in elems:
            pool[e] = sorted(pool[e], key=_key)
        for _ in range(6):
            a, b = _orset(rng, elems, pool), _orset(rng, elems, pool)
            for op, case in ((MERGE, (MERGE, OK, 0, _tb(a), _tb(b), _tb(oorset.merge(a, b)))),
                             (VALUE, (VALUE, OK, 0, _tb(a), b"", _tb(oorset.value(a)))),
                             (SINFL, (SINFL, OK, int(olat.is_strict_inflation(
                                 "lasp_orset", a, oorset.merge(a, b))), _tb(a),
                                 _tb(oorset.merge(a, b)), b""))):
                _check(case, _run_case(ctx, case))
        assert ctx.nif_stats()["host_encoded_passes"] > 0
    finally:
        ctx.close()


@pytest.mark.gpu
def test_nif_flags_in_other_atom_encodings_and_second_copy():
    """Operands whose flags use SMALL_ATOM_UTF8_EXT (an OTP 26 node's term_to_binary):
    decoded alike; the answer is written with ATOM_EXT flags, one byte longer per token,
    so it outgrows the first copy's bound and takes the second copy."""
    ctx = _ctx()
    try:
        rng = random.Random(9)
        toks = sorted(_tokens(rng, 3000))

        def utf8_flags(img: bytes) -> bytes:
            return img.replace(bytes([100, 0, 4]) + b"true", bytes([119, 4]) + b"true") \
                      .replace(bytes([100, 0, 5]) + b"false", bytes([119, 5]) + b"false")

        a = [(e, [(toks[3 * e + j], bool(j % 2)) for j in range(3)]) for e in range(0, 1000, 2)]
        b = [(e, [(toks[3 * e + j], bool(j % 2)) for j in range(3)]) for e in range(1, 1000, 2)]
        ia, ib = utf8_flags(_tb(a)), utf8_flags(_tb(b))
        assert len(ia) < len(_tb(a))
        v, img = ctx.nif_merge(ia, ib)
        assert v == OK and img == _tb(oorset.merge(a, b))
        assert len(img) > len(ia) + len(ib)
    finally:
        ctx.close()


@pytest.mark.gpu
def test_nif_four_schedulers_python_threads():
    """Four threads, one context each, the same cases in different orders (ctypes drops
    the GIL inside each call, so the calls overlap on the device)."""
    cases = valid_cases(seed=21, n=12) + fallback_cases(seed=22)
    errors = []

    def worker(tid):
        try:
            ctx = _ctx()
            try:
                for r in range(3):
                    for k in range(len(cases)):
                        case = cases[(k + 13 * tid + 5 * r) % len(cases)]
                        _check(case, _run_case(ctx, case))
            finally:
                ctx.close()
        except Exception as e:          # noqa: BLE001 — reported below
            errors.append((tid, repr(e)))

    ths = [threading.Thread(target=worker, args=(t,)) for t in range(4)]
    for t in ths:
        t.start()
    for t in ths:
        t.join(timeout=240)
    assert not any(t.is_alive() for t in ths)
    assert not errors, errors


@pytest.mark.gpu
def test_nif_four_schedulers_plain_c(tmp_path):
    """tests/c/laspj_nif_threads.c: 4 pthreads x 4 contexts through laspj.h alone,
    verdicts / booleans / images compared with the oracle's answers byte for byte."""
    exe = _build_threads_exe(tmp_path)
    p = tmp_path / "cases.bin"
    write_cases(p, valid_cases(seed=31, n=16) + fallback_cases(seed=32))
    res = subprocess.run([exe, str(p), "4"], capture_output=True, text=True, timeout=240)
    assert res.returncode == 0, res.stdout + res.stderr
    assert "laspj NIF threads OK" in res.stdout


# ------------------------------------------------------------------ `==` classes

def _oracle_answer(op, a, b):
    """The reference's answer for (op, terms a, b) from the oracle."""
    if op == MERGE:
        return _tb(oorset.merge(a, b))
    if op == VALUE:
        return _tb(oorset.value(a))
    if op == EQUAL:
        return oorset.equal(a, b)
    return olat.is_inflation("lasp_orset", a, b) if op == INFL else \
        olat.is_strict_inflation("lasp_orset", a, b)


def equal_term_cases(seed=3):
    """Operands holding `==`-equal terms under other images (1 / 1.0 as elements, inside
    tuples and lists, as tokens), in both orders and after the other image registered."""
    rng = random.Random(seed)
    t = _tokens(rng, 8)
    pairs = [
        ([(1, [(t[0], False)])], [(1.0, [(t[1], False)])]),
        ([(1.0, [(t[0], True)])], [(1, [(t[0], False)])]),
        ([((Atom("a"), 1), [(t[2], False)])], [((Atom("a"), 1.0), [(t[3], True)])]),
        ([([1, 2], [(t[4], False)])], [([1.0, 2], [(t[4], False)])]),
        ([(5, [(7, False)])], [(5, [(7.0, True)])]),
        ([(2, [(t[5], False)]), (3, [(t[6], False)])], [(3.0, [(t[6], True)])]),
    ]
    out = []
    for a, b in pairs:
        for op in (MERGE, EQUAL, INFL, SINFL):
            out.append((op, a, b))
            out.append((op, b, a))
        out.append((VALUE, b, None))
    return out


@pytest.mark.gpu
def test_nif_equal_terms_answer_the_oracle_or_fallback():
    """`1` and `1.0` (and terms holding them, and tokens) are
    one orddict key for the reference (orddict:merge's equal clause keeps the left key,
    lasp_orset.erl:128-134; equal/2 is ==, :136-138).  The dictionary refuses the second
    image of a `==` class (LASPJ_DEC_EQUAL_TERMS), so every such call answers the oracle's
    term or FALLBACK (the reference's own clause) — never a two-key answer with verdict OK.
    The context keeps answering ordinary calls afterwards."""
    ctx = _ctx()
    try:
        n_fb = 0
        for op, a, b in equal_term_cases():
            got = _run_case(ctx, (op, None, None, _tb(a), _tb(b) if b is not None else b"", b""))
            v, ans = got
            if v == FALLBACK:
                n_fb += 1
                assert ans is None
                continue
            assert v == OK
            want = _oracle_answer(op, a, b)
            assert ans == want, (op, a, b, ans, want)
        assert n_fb >= 20
        for case in valid_cases(seed=4, n=6):
            _check(case, _run_case(ctx, case))
    finally:
        ctx.close()


@pytest.mark.gpu
def test_nif_unresolved_call_answers_fallback():
    """run()'s post-condition: a call whose device passes run out
    before its statuses are final answers FALLBACK, not the superseded pass's answer.  With
    one pass allowed (LASPJ_TUNE_NIF_PASSES), a merge that meets a fresh token registers it
    and has no pass left: FALLBACK; the same call with the default passes answers the
    oracle's merge."""
    from lasp_amd import _lib
    ctx = _ctx()
    try:
        rng = random.Random(12)
        elems, pool = _universe(rng, 40)
        a, b = _orset(rng, elems, pool), _orset(rng, elems, pool)
        assert ctx.nif_merge(_tb(a), _tb(b)) == (OK, _tb(oorset.merge(a, b)))
        ctx.set_tuning(_lib.TUNE_NIF_PASSES, 1)
        e = [x for x, _ts in b][0]
        b2 = oorset.merge(b, [(e, [(b"\x07" * 20, False)])])
        assert ctx.nif_merge(_tb(a), _tb(b2)) == (FALLBACK, None)
        # (now registered: one pass is enough)
        assert ctx.nif_merge(_tb(a), _tb(b2)) == (OK, _tb(oorset.merge(a, b2)))
        b3 = oorset.merge(b, [(e, [(b"\x08" * 20, True)])])
        assert ctx.nif_merge(_tb(a), _tb(b3)) == (FALLBACK, None)
        ctx.set_tuning(_lib.TUNE_NIF_PASSES, 0)
        b4 = oorset.merge(b, [(e, [(b"\x09" * 20, True)])])
        assert ctx.nif_merge(_tb(a), _tb(b4)) == (OK, _tb(oorset.merge(a, b4)))
    finally:
        ctx.close()


@pytest.mark.gpu
def test_nif_merge_of_unseen_binary_tokens():
    """merge/2 of a known state and one carrying tokens the context has not seen (another
    node's updates, lasp_orset.erl:222-230): the decoders take them in the first pass, the
    images are patched, and a second launch only joins and writes (no staging or decode
    again); both operands carrying the same new token keep it once; two different new
    tokens given one slot by the two operands decode the usual way.  Every answer is the
    oracle's."""
    ctx = _ctx()
    try:
        rng = random.Random(71)
        rb = lambda b: bytes([b]) + bytes(rng.getrandbits(8) for _ in range(19))  # noqa: E731
        base = [(e, sorted([(rb(0x40 + 2 * k), k == 1) for k in range(2)], key=_key))
                for e in range(3000)]
        assert ctx.nif_merge(_tb(base), _tb(base)) == (OK, _tb(base))
        for case in ("one side", "both sides alike", "both sides differ"):
            picks = sorted(rng.sample(range(3000), 25))
            new = {e: [rb(rng.choice((0x00, 0x41, 0xff)))] for e in picks}
            b = [(e, sorted(ts + [(t, False) for t in new.get(e, [])], key=_key))
                 for e, ts in base]
            if case == "one side":
                a = base
            elif case == "both sides alike":
                a = b
            else:
                other = {e: [rb(0x43)] for e in picks}
                a = [(e, sorted(ts + [(t, True) for t in other.get(e, [])], key=_key))
                     for e, ts in base]
            s0 = ctx.nif_stats()
            assert ctx.nif_merge(_tb(a), _tb(b)) == (OK, _tb(oorset.merge(a, b))), case
            s1 = ctx.nif_stats()
            if case != "both sides differ":
                assert s1["device_new_tokens"] - s0["device_new_tokens"] == 25, case
                assert s1["device_passes"] - s0["device_passes"] == 2, case
            assert s1["fallbacks"] == s0["fallbacks"]
            # the same merge again: every token known, one pass
            assert ctx.nif_merge(_tb(a), _tb(b)) == (OK, _tb(oorset.merge(a, b)))
            assert ctx.nif_stats()["device_passes"] - s1["device_passes"] == 1
            base = oorset.merge(a, b)
    finally:
        ctx.close()
