"""Wire codec: to_binary / from_binary (src/lasp_orset.erl:198-214, src/lasp_gset.erl:
111-128; riak_dt:to_binary/1 = term_to_binary).

CPU: the oracle's external-term-format restatement against the format's published
examples; the host fragment encoder / decoder against the oracle.  GPU: payloads the
device assembles from cells, byte for byte against the oracle, on the golden-vector
states, random states with mixed terms, and a large synthetic batch; and the
reference's round-trip property from_binary(to_binary(S)) == S
(test/crdt_statem_eqc.erl:108-121).
"""

import contextlib
import json
import os
import random

import pytest
from hypothesis import given, settings, strategies as st

from oracle import etf as oetf
from lasp_amd.terms import Atom as PAtom
from oracle.terms import Atom, exact_eq

SOAK = int(__import__("os").environ.get("LASPJ_SOAK", "1"))   # x examples for a soak run

HERE = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")

# (term, term_to_binary(term)) from the external term format specification
PUBLISHED = [
    (1, bytes([131, 97, 1])),
    (255, bytes([131, 97, 255])),
    (256, bytes([131, 98, 0, 0, 1, 0])),
    (-1, bytes([131, 98, 255, 255, 255, 255])),
    (1 << 40, bytes([131, 110, 6, 0, 0, 0, 0, 0, 0, 1])),
    (-(1 << 40), bytes([131, 110, 6, 1, 0, 0, 0, 0, 0, 1])),
    (1.5, bytes([131, 70, 63, 248, 0, 0, 0, 0, 0, 0])),
    (True, bytes([131, 100, 0, 4]) + b"true"),
    (False, bytes([131, 100, 0, 5]) + b"false"),
    (Atom("a"), bytes([131, 100, 0, 1, 97])),
    (b"a", bytes([131, 109, 0, 0, 0, 1, 97])),
    ((Atom("a"), 1), bytes([131, 104, 2, 100, 0, 1, 97, 97, 1])),
    ([], bytes([131, 106])),
    ([1, 2], bytes([131, 107, 0, 2, 1, 2])),
    ([256], bytes([131, 108, 0, 0, 0, 1, 98, 0, 0, 1, 0, 106])),
    ([(1, [(b"t", False)])], bytes([131, 108, 0, 0, 0, 1, 104, 2, 97, 1, 108, 0, 0, 0, 1,
                                    104, 2, 109, 0, 0, 0, 1, 116, 100, 0, 5]) + b"false"
     + bytes([106, 106])),
]


@pytest.mark.parametrize("term,image", PUBLISHED)
def test_oracle_published_examples(term, image):
    assert oetf.term_to_binary(term) == image
    assert exact_eq(oetf.binary_to_term(image), term)


def test_oracle_compressed_roundtrip_and_errors():
    big = [(k, [(bytes([k % 251]) * 20, False)]) for k in range(300)]
    z = oetf.term_to_binary(big, compressed=1)
    assert z[:2] == bytes([131, 80]) and len(z) < len(oetf.term_to_binary(big))
    assert exact_eq(oetf.binary_to_term(z), big)
    for bad in (b"", b"\x83", b"\x84\x61\x01", b"\x83\x61\x01\x00", b"\x83\x6c\x00\x00\x00\x01"):
        with pytest.raises(ValueError):
            oetf.binary_to_term(bad)


_atoms = st.sampled_from([Atom("a"), Atom("undefined"), Atom("ok"), True, False,
                          Atom("été")])
_leaf = st.one_of(st.integers(-(1 << 70), 1 << 70), st.integers(0, 300), _atoms,
                  st.binary(max_size=40), st.floats(allow_nan=False, allow_infinity=False))
_terms = st.recursive(_leaf, lambda ch: st.one_of(st.lists(ch, max_size=5),
                                                  st.tuples(ch, ch), st.tuples(ch)),
                      max_leaves=12)


@settings(max_examples=400 * SOAK, deadline=None)
@given(_terms)
def test_host_encoder_matches_oracle(t):
    from lasp_amd import etf
    img = etf.encode(t)
    assert bytes([131]) + img == oetf.term_to_binary(t)
    assert exact_eq(etf.binary_to_term(bytes([131]) + img), oetf.binary_to_term(bytes([131]) + img))


def test_host_decoder_rejects_malformed():
    from lasp_amd import etf
    for bad in (b"", b"\x83", b"\x83\x62\x00", b"\x83\x6c\x00\x00\x00\x01\x61\x01\x61",
                b"\x83\x61\x01\x00", b"\x83\xff"):
        with pytest.raises(ValueError):
            etf.binary_to_term(bad)


def test_domain_etf_arrays_slice_the_images():
    from lasp_amd import etf
    from lasp_amd.codec import Domain
    s = [(1, [(b"x" * 20, False), (b"a" * 20, True)]), (PAtom("b"), [(b"q" * 3, False)]),
         ((1, 2), [(b"z" * 20, True)])]
    dom = Domain()
    dom.register_orset(s)
    eb, eo, order, tb, to, tord = dom.etf_arrays(5)
    assert [dom.elements.terms[i] for i in order[:3]] == [1, PAtom("b"), (1, 2)]
    assert list(order[3:]) == [3, 4]
    for es, term in enumerate(dom.elements.terms):
        assert eb[eo[es]:eo[es + 1]] == etf.encode(term)
    assert eo[4] == eo[5] == eo[3]                       # unused slots: empty images
    e0 = dom.element_slot(1, create=False)
    assert list(tord[64 * e0:64 * e0 + 3]) == [1, 0, 0xFF]   # b"aaa.." < b"xxx.."
    for k in (0, 1):
        t = dom.tokens[e0].terms[k]
        assert tb[to[64 * e0 + k]:to[64 * e0 + k + 1]] == etf.encode(t)


def test_from_binary_errors_and_tags():
    from lasp_amd import etf, gset, orset
    s = [(1, [(b"t" * 20, False)])]
    payload = oetf.to_binary(etf.DT_ORSET_TAG, 1, s)
    assert exact_eq(orset.from_binary(payload), s)
    assert orset.from_binary(bytes([etf.DT_ORSET_TAG, 2]) + payload[2:]) == \
        ("error", "unsupported_version", 2)
    assert orset.from_binary(b"\x00\x01\x83\x6a") == ("error", "invalid_binary")
    assert orset.to_binary2(2, s) == ("error", "unsupported_version", 2)
    g = oetf.to_binary(etf.DT_GSET_TAG, 1, [1, 2, 3])
    assert gset.from_binary(g) == ("ok", [1, 2, 3])
    assert orset.from_binary(oetf.to_binary(etf.DT_ORSET_TAG, 1, s, compressed=1)) == s


# ------------------------------------------------------------------ GPU

def _golden(name):
    from tests.golden.termjson import dec
    with open(os.path.join(HERE, name)) as f:
        cases = json.load(f)["cases"]
    return [dec(c[k], PAtom) for c in cases for k in ("a", "b")]


@pytest.mark.gpu
def test_gpu_orset_to_binary_golden():
    from lasp_amd import etf, orset
    for s in _golden("orset_cases.json"):
        got = orset.to_binary(s)
        assert got == oetf.to_binary(etf.DT_ORSET_TAG, 1, s), s
        assert exact_eq(orset.from_binary(got), s)


@pytest.mark.gpu
def test_gpu_gset_to_binary_golden():
    from lasp_amd import etf, gset
    states = _golden("gset_cases.json") + [[], [0, 1, 255], [1, 256], list(range(300)),
                                           [PAtom("a"), (1, 2), b"x"]]
    for s in states:
        got = gset.to_binary(s)
        assert got == oetf.to_binary(etf.DT_GSET_TAG, 1, s), s
        back = gset.from_binary(got)
        assert back[0] == "ok" and exact_eq(back[1], s)


def _random_orsets(rng, n, mixed):
    elems = list(range(0, 600, 7)) + ([PAtom("x"), (1, PAtom("y")), b"bin", 1 << 40, -5, 2.5]
                                      if mixed else [])
    # each element draws its tokens from a pool of 40 (a dictionary holds <= 64 per element)
    pool = {hk: [bytes(rng.randrange(256) for _ in range(20 if not mixed else rng.choice([1, 20, 33])))
                 for _ in range(40)] for hk in range(len(elems))}
    out = []
    for _ in range(n):
        d = {}
        for i in rng.sample(range(len(elems)), rng.randint(0, min(40, len(elems)))):
            d[elems[i]] = {t: rng.random() < 0.3 for t in rng.sample(pool[i], rng.randint(1, 6))}
        out.append(d)
    from oracle.otp import lists_sort
    res = []
    for d in out:
        keys = lists_sort(list(d.keys()))
        res.append([(k, [(t, d[k][t]) for t in sorted(d[k])]) for k in keys])
    return res


@pytest.mark.gpu
@pytest.mark.parametrize("mixed", [False, True])
def test_gpu_orset_batch_payloads_random(mixed):
    """One batch of 300 replicas over one dictionary; uniform (20-byte tokens) and
    mixed token / element images; bare term_to_binary images and tagged payloads."""
    from lasp_amd import engine, etf
    from lasp_amd.codec import Domain
    from lasp_amd.orset import context
    rng = random.Random(7 + mixed)
    states = _random_orsets(rng, 300, mixed)
    dom = Domain()
    for s in states:
        dom.register_orset(s)
    E = dom.size + 3                                     # unused trailing slots
    b = context().orset_batch(len(states), E)
    b.upload(dom.encode_orset(states, E))
    d = engine.ETFDict(context(), E, *dom.etf_arrays(E))
    bare = b.to_binaries(d)
    tagged = b.to_binaries(d, tag=etf.DT_ORSET_TAG, vers=1)
    for s, x, y in zip(states, bare, tagged):
        assert x == oetf.term_to_binary(s)
        assert y == bytes([etf.DT_ORSET_TAG, 1]) + x


@pytest.mark.gpu
def test_gpu_etf_rejects_unregistered_slots():
    from lasp_amd import _lib, engine
    from lasp_amd.codec import Domain
    from lasp_amd.orset import context
    s = [(1, [(b"t" * 20, False)])]
    dom = Domain()
    dom.register_orset(s)
    b = context().orset_batch(2, 4)
    cells = dom.encode_orset([s, s], 4)
    cells[1, 2, 0] = 1                                   # element slot 2 has no image
    b.upload(cells)
    d = engine.ETFDict(context(), 4, *dom.etf_arrays(4))
    with pytest.raises(_lib.LaspjError):
        b.etf_encode(d)
    cells[1, 2, 0] = 0
    cells[1, 0, 0] = 0b10                                # token slot 1 of element 0
    b.upload(cells)
    with pytest.raises(_lib.LaspjError):
        b.etf_encode(d)


@pytest.mark.gpu
def test_gpu_orset_large_synthetic_batch():
    """4096 replicas x 512 slots x 64 token slots (seeded synthetic cells, the bench
    dictionary of 20-byte tokens): sampled replicas match the oracle byte for byte and
    the offsets are the prefix sums of the oracle's payload sizes."""
    import numpy as np
    from lasp_amd import engine, etf
    from lasp_amd.codec import Domain
    from lasp_amd.orset import context
    from oracle import columnar as orc
    R, E = 4096, 512
    b = context().orset_batch(R, E)
    b.fill_synthetic(5)
    toks = orc.synth_tokens(E)
    dom = Domain()
    for e in range(E):
        es = dom.element_slot(e)
        for k in range(64):
            dom.token_slot(es, bytes(toks[e][k]))
    d = engine.ETFDict(context(), E, *dom.etf_arrays(E))
    offs, out, total = b.etf_encode(d, tag=etf.DT_ORSET_TAG, vers=1)
    o = offs.download(np.uint64)
    cells = b.download()
    assert o[0] == 0 and int(o[-1]) == total
    for i in list(range(0, R, 257)) + [R - 1]:
        s = dom.decode_orset(cells[i])
        want = oetf.to_binary(etf.DT_ORSET_TAG, 1, s)
        got = out.download(np.uint8, count=int(o[i + 1] - o[i]), offset=int(o[i])).tobytes()
        assert got == want, i


def _etf_variants(ctx, fn, knobs=(0, 1, 2, 3, 4, 5)):
    """fn() under the record kernel (LASPJ_TUNE_ETF_KERNEL 0, chosen for uniform token
    images: records per element thread when <= 8 token slots, else spread over lanes),
    the element-staging kernels (1) and the lane-spread record kernel at other window
    sizes (2, 3: 16 and 20 KiB) and at 24 KiB (4), and the per-element-thread record
    kernel for any token count (5)."""
    from lasp_amd._lib import TUNE_ETF_KERNEL
    out = []
    try:
        for k in knobs:
            ctx.set_tuning(TUNE_ETF_KERNEL, k)
            out.append(fn())
    finally:
        ctx.set_tuning(TUNE_ETF_KERNEL, 0)
    return out


@pytest.mark.gpu
@pytest.mark.parametrize("tok_len,long_elems,pool_n", [
    (20, False, 64), (20, True, 64), (41, True, 64), (42, False, 64), (1, True, 64),
    (20, True, 6), (41, False, 8), (1, False, 3)])
def test_gpu_orset_record_kernel_edges(tok_len, long_elems, pool_n):
    """Payloads crossing many 16 KiB windows (up to 300 elements x 64 tokens), empty and
    one-token replicas, element images longer than the 48-byte fast header (binaries,
    tuples, long atoms), token images at the record kernel's 48-byte limit (41-byte
    binaries) and just past it (42: the staging kernels), E not a multiple of 256,
    elements with up to 64 token slots (records spread over lanes) and with <= 8 (records
    staged by their element's thread): every kernel matches the oracle byte for byte,
    bare and tagged."""
    from lasp_amd import engine, etf
    from lasp_amd.codec import Domain
    from lasp_amd.orset import context
    from oracle.otp import lists_sort
    rng = random.Random(tok_len * 7 + long_elems)
    elems = list(range(0, 900, 3))
    if long_elems:
        elems += [b"L" * 60, (PAtom("k"), b"v" * 50), PAtom("a" * 47), b"s" * 40, 1 << 70]
    pool = {i: [bytes(rng.randrange(256) for _ in range(tok_len)) for _ in range(pool_n)]
            for i in range(len(elems))}
    if tok_len == 1:                                  # distinct one-byte tokens
        pool = {i: [bytes([x]) for x in rng.sample(range(256), pool_n)]
                for i in range(len(elems))}
    raw = [{}, {elems[5]: {pool[5][0]: False}},
           {elems[i]: {t: rng.random() < 0.25 for t in pool[i]} for i in range(len(elems))}]
    for _ in range(37):
        d = {}
        k = rng.choice([1, 3, 40, 150, len(elems)])
        for i in rng.sample(range(len(elems)), k):
            d[elems[i]] = {t: rng.random() < 0.3
                           for t in rng.sample(pool[i], rng.randint(1, pool_n))}
        raw.append(d)
    states = []
    for d in raw:
        states.append([(k, [(t, d[k][t]) for t in sorted(d[k])]) for k in lists_sort(list(d))])
    dom = Domain()
    for s in states:
        dom.register_orset(s)
    E = dom.size + 11
    ctx = context()
    b = ctx.orset_batch(len(states), E)
    b.upload(dom.encode_orset(states, E))
    d = engine.ETFDict(ctx, E, *dom.etf_arrays(E))
    for bare, tagged in _etf_variants(ctx, lambda: (b.to_binaries(d),
                                                    b.to_binaries(d, tag=etf.DT_ORSET_TAG))):
        for s, x, y in zip(states, bare, tagged):
            assert x == oetf.term_to_binary(s)
            assert y == bytes([etf.DT_ORSET_TAG, 1]) + x


@pytest.mark.gpu
@pytest.mark.parametrize("R,nelem,pool_n,density", [
    (1, 3000, 64, 0.9), (3, 2600, 6, 0.5), (2, 5000, 40, 0.02), (200, 3000, 3, 0.08)])
def test_gpu_record_kernel_split_payloads(R, nelem, pool_n, density):
    """Few long payloads (the NIF's one merged value): the writer's split mode gives each
    block a run of 256-element chunks of one payload at its chunk's byte offset — one to
    200 payloads of up to 5000 elements, dense and sparse (whole chunks empty), 64 and
    <= 8 token slots per element, element images across chunk edges: every payload equals
    the oracle's term_to_binary byte for byte, bare and tagged, under every writer."""
    from lasp_amd import engine, etf
    from lasp_amd.codec import Domain
    from lasp_amd.orset import context
    from oracle.otp import lists_sort
    rng = random.Random(R * 131 + nelem)
    elems = list(range(nelem))
    pool = [bytes(rng.randrange(256) for _ in range(20)) for _ in range(97)]
    states = []
    for i in range(R):
        d = {}
        for e in elems:
            if rng.random() < density:
                d[e] = {pool[(e * 7 + j) % 97]: rng.random() < 0.3
                        for j in rng.sample(range(pool_n), rng.randint(1, min(pool_n, 6)))}
        states.append([(k, [(t, d[k][t]) for t in sorted(d[k])]) for k in lists_sort(list(d))])
    dom = Domain()
    for e in elems:                                   # every element registered, in order
        es = dom.element_slot(e)
        for j in range(pool_n):
            dom.token_slot(es, pool[(e * 7 + j) % 97])
    E = dom.size
    ctx = context()
    b = ctx.orset_batch(R, E)
    b.upload(dom.encode_orset(states, E))
    d = engine.ETFDict(ctx, E, *dom.etf_arrays(E))
    want = [oetf.term_to_binary(s) for s in states]
    for bare, tagged in _etf_variants(ctx, lambda: (b.to_binaries(d),
                                                    b.to_binaries(d, tag=etf.DT_ORSET_TAG))):
        assert bare == want
        assert tagged == [bytes([etf.DT_ORSET_TAG, 1]) + w for w in want]


@pytest.mark.gpu
def test_gpu_etf_split_sizes_reject_unregistered_slots():
    """The chunked size pass (few long payloads) flags a present slot without an image
    like the per-payload one, and agrees with it on valid payloads."""
    import numpy as np
    from lasp_amd import _lib, engine
    from lasp_amd.codec import Domain
    from lasp_amd.orset import context
    n = 3000
    s = [(e, [(b"t" + e.to_bytes(19, "big"), e % 3 == 0)]) for e in range(n)]
    dom = Domain()
    dom.register_orset(s)
    ctx = context()
    b = ctx.orset_batch(1, n + 5)
    cells = dom.encode_orset([s], n + 5)
    b.upload(cells)
    d = engine.ETFDict(ctx, n + 5, *dom.etf_arrays(n + 5))
    offs, out, total = b.etf_encode(d)
    assert int(offs.download(np.uint64)[1]) == total == len(oetf.term_to_binary(s))
    cells[0, n + 2, 0] = 1                               # slot n + 2 has no image
    b.upload(cells)
    with pytest.raises(_lib.LaspjError):
        b.etf_encode(d)
    cells[0, n + 2, 0] = 0
    cells[0, 17, 0] = 0b100                              # token slot 2 of element 17
    b.upload(cells)
    with pytest.raises(_lib.LaspjError):
        b.etf_encode(d)


@pytest.mark.gpu
def test_gpu_record_kernel_whole_buffer_equals_staging():
    """2048 replicas x 512 slots x 64 token slots (~1.1 GB of payloads): the record and
    the staging kernels write identical buffers, every byte of every replica."""
    import numpy as np
    from lasp_amd import engine, etf
    from lasp_amd.codec import Domain
    from lasp_amd.orset import context
    from oracle import columnar as orc
    R, E = 2048, 512
    ctx = context()
    b = ctx.orset_batch(R, E)
    b.fill_synthetic(11)
    toks = orc.synth_tokens(E)
    dom = Domain()
    for e in range(E):
        es = dom.element_slot(e * 1000)
        for k in range(64):
            dom.token_slot(es, bytes(toks[e][k]))
    d = engine.ETFDict(ctx, E, *dom.etf_arrays(E))

    def run():
        offs, out, total = b.etf_encode(d, tag=etf.DT_ORSET_TAG, vers=1)
        return offs.download(np.uint64), out.download(np.uint8, count=total)
    (o1, p1), *rest = _etf_variants(ctx, run)
    for o2, p2 in rest:
        assert np.array_equal(o1, o2)
        assert np.array_equal(p1, p2)


@pytest.mark.gpu
def test_gpu_record_kernel_runs_with_tiny_payloads():
    """6000 replicas (several per block run): empty payloads (2 / 4 bytes), one-token
    payloads shorter than 16 bytes of element data, and larger ones, interleaved — the
    carry flows through payloads smaller than a 16-byte chunk; every payload equals the
    oracle's, bare and tagged, under every writer variant."""
    from lasp_amd import engine, etf
    from lasp_amd.codec import Domain
    from lasp_amd.orset import context
    from oracle.otp import lists_sort
    rng = random.Random(99)
    toks = [bytes(rng.randrange(256) for _ in range(20)) for _ in range(12)]
    states = []
    for i in range(6000):
        kind = rng.random()
        d = {}
        if kind < 0.4:
            pass                                              # empty
        elif kind < 0.8:
            d[rng.randrange(5)] = {toks[rng.randrange(12)]: rng.random() < 0.5}
        else:
            for e in rng.sample(range(40), rng.randint(2, 30)):
                d[e] = {t: rng.random() < 0.3 for t in rng.sample(toks, rng.randint(1, 12))}
        states.append([(k, [(t, d[k][t]) for t in sorted(d[k])]) for k in lists_sort(list(d))])
    dom = Domain()
    for s in states:
        dom.register_orset(s)
    E = dom.size
    ctx = context()
    b = ctx.orset_batch(len(states), E)
    b.upload(dom.encode_orset(states, E))
    d = engine.ETFDict(ctx, E, *dom.etf_arrays(E))
    want = [oetf.term_to_binary(s) for s in states]
    for bare, tagged in _etf_variants(ctx, lambda: (b.to_binaries(d),
                                                    b.to_binaries(d, tag=etf.DT_ORSET_TAG))):
        assert bare == want
        assert tagged == [bytes([etf.DT_ORSET_TAG, 1]) + w for w in want]


@contextlib.contextmanager
def _read_kernel(ctx, knob):
    """LASPJ_TUNE_ETF_READ for the duration: 0 = batched records (+ element batches at
    <= 8 token slots, and for small elements of many-token dictionaries), 1 = serial
    scan, 2 = batched records only, 7 = no many-token element batches, 8 = the same as
    0, 11..15 = the G-Set decoder's one-wave forms, never split (the OR-Set decoders as
    with 0), 4 = every payload
    longer than 256 bytes split between waves (segment mode: header search, chain check, redo
    of failed replicas); "seg512": the default kernels with every payload longer than 512
    bytes split (LASPJ_TUNE_ETF_SEG)."""
    from lasp_amd import _lib
    if knob == "seg512":
        ctx.set_tuning(_lib.TUNE_ETF_SEG, 512)
    else:
        ctx.set_tuning(_lib.TUNE_ETF_READ, knob)
    try:
        yield
    finally:
        ctx.set_tuning(_lib.TUNE_ETF_READ, 0)
        ctx.set_tuning(_lib.TUNE_ETF_SEG, 0)


def _decode_setup(states, rng_seed=0):
    from lasp_amd import engine
    from lasp_amd.codec import Domain
    from lasp_amd.orset import context
    dom = Domain()
    for s in states:
        dom.register_orset(s)
    E = dom.size + 5
    ctx = context()
    d = engine.ETFDict(ctx, E, *dom.etf_arrays(E))
    return ctx, dom, E, d


def _upload_payloads(ctx, blobs):
    import numpy as np
    off = np.zeros(len(blobs) + 1, np.uint64)
    off[1:] = np.cumsum([len(b) for b in blobs])
    flat = b"".join(blobs) or b"\0"
    pay = ctx.buffer(len(flat))
    pay.upload(np.frombuffer(flat, np.uint8))
    offs = ctx.buffer(8 * len(off))
    offs.upload(off)
    return pay, offs


@pytest.mark.gpu
@pytest.mark.parametrize("knob", [0, 1, 4, "seg512"])
@pytest.mark.parametrize("tagged", [False, True])
def test_gpu_from_binary_round_trip(tagged, knob):
    """Device from_binary/1 of oracle payloads (term_to_binary of random orddicts with
    20-byte tokens, long and short element terms) yields the same cells the host
    encoder gives, and device to_binary -> from_binary is the identity on cells."""
    import numpy as np
    from lasp_amd import _lib, etf
    rng = random.Random(31 + tagged)
    states = _random_orsets(rng, 200, mixed=False)
    states += [[], [((PAtom("k"), b"v" * 50), [(b"t" * 20, True)])],
               [(1 << 70, [(b"u" * 20, False), (b"w" * 20, True)])]]
    ctx, dom, E, d = _decode_setup(states)
    tag = etf.DT_ORSET_TAG if tagged else -1
    blobs = [oetf.to_binary(tag, 1, s) if tagged else oetf.term_to_binary(s) for s in states]
    pay, offs = _upload_payloads(ctx, blobs)
    b = ctx.orset_batch(len(states), E)
    with _read_kernel(ctx, knob):
        st = b.etf_decode(d, pay, offs, tag=tag, vers=1)
        assert (st == _lib.DEC_OK).all(), np.nonzero(st)[0][:10]
        want = dom.encode_orset(states, E)
        assert np.array_equal(b.download(), want)
        # device to_binary -> from_binary
        offs2, out2, _ = b.etf_encode(d, tag=tag, vers=1)
        b2 = ctx.orset_batch(len(states), E)
        assert (b2.etf_decode(d, out2, offs2, tag=tag, vers=1) == 0).all()
        assert np.array_equal(b2.download(), want)


@pytest.mark.gpu
@pytest.mark.parametrize("tok_len", [1, 9, 10, 20, 21, 22, 41])
@pytest.mark.parametrize("pool_n", [3, 40])
def test_gpu_from_binary_record_lengths(tok_len, pool_n):
    """Records 104 2 <binary> of 8 .. 48 bytes (token binaries of 1 .. 41 bytes) on both
    sides of the decoder's compare paths (<= 16, <= 28 and longer record templates),
    with few token slots per element (element batches) and many (record locator):
    from_binary of the oracle's payloads gives the encoder's cells."""
    import numpy as np
    from lasp_amd import _lib
    from oracle.otp import lists_sort
    rng = random.Random(tok_len * 13 + pool_n)
    elems = list(range(0, 400, 3))
    pool = {i: list({bytes(rng.randrange(256) for _ in range(tok_len)) for _ in range(pool_n)})
            for i in range(len(elems))}
    if tok_len == 1:
        pool = {i: [bytes([x]) for x in rng.sample(range(256), pool_n)] for i in range(len(elems))}
    states = [[]]
    for _ in range(60):
        d = {}
        for i in rng.sample(range(len(elems)), rng.choice([1, 5, 60, len(elems)])):
            d[elems[i]] = {t: rng.random() < 0.3 for t in rng.sample(pool[i], rng.randint(1, len(pool[i])))}
        states.append([(k, [(t, d[k][t]) for t in sorted(d[k])]) for k in lists_sort(list(d))])
    ctx, dom, E, d = _decode_setup(states)
    blobs = [oetf.term_to_binary(s) for s in states]
    pay, offs = _upload_payloads(ctx, blobs)
    want = dom.encode_orset(states, E)
    for knob in (0, "seg512"):
        b = ctx.orset_batch(len(states), E)
        with _read_kernel(ctx, knob):
            st = b.etf_decode(d, pay, offs, tag=-1, vers=1)
        assert (st == _lib.DEC_OK).all(), (knob, np.nonzero(st)[0][:10])
        assert np.array_equal(b.download(), want), knob


@pytest.mark.gpu
@pytest.mark.parametrize("knob", [0, 1, 2, 4, 6, "seg512"])
def test_gpu_from_binary_errors_and_atom_forms(knob):
    """Statuses: ?INVALID_BINARY (wrong tag, no 131, empty), ?UNSUPPORTED_VERSION,
    malformed (truncated, trailing byte, bad flag atom, element without tokens), terms
    outside the dictionary or out of term order; SMALL_ATOM_UTF8_EXT / ATOM_UTF8_EXT
    flags (what newer OTP releases emit) decode like ATOM_EXT.  No payload faults."""
    import numpy as np
    from lasp_amd import _lib, etf
    tok = [bytes([k]) * 20 for k in range(1, 6)]
    s0 = [(1, [(tok[0], False), (tok[1], True)]), (2, [(tok[2], False)])]
    ctx, dom, E, d = _decode_setup([s0, [(3, [(tok[3], True)])]])
    T = etf.DT_ORSET_TAG
    good = oetf.to_binary(T, 1, s0)
    small_atoms = good.replace(bytes([100, 0, 4]) + b"true", bytes([119, 4]) + b"true") \
                      .replace(bytes([100, 0, 5]) + b"false", bytes([119, 5]) + b"false")
    utf8_atoms = good.replace(bytes([100, 0, 4]) + b"true", bytes([118, 0, 4]) + b"true")
    unknown = oetf.to_binary(T, 1, [(1, [(b"z" * 20, False)])])
    out_of_order = oetf.to_binary(T, 1, [(2, [(tok[2], False)]), (1, [(tok[0], False)])])
    no_tokens = oetf.to_binary(T, 1, [(1, [])])
    bad_flag = good.replace(b"false", b"fals\x65"[:4] + b"x", 1)
    cases = [
        (good, _lib.DEC_OK), (small_atoms, _lib.DEC_OK), (utf8_atoms, _lib.DEC_OK),
        (bytes([T + 1]) + good[1:], _lib.DEC_INVALID_BINARY),
        (bytes([T, 2]) + good[2:], _lib.DEC_UNSUPPORTED_VERSION),
        (b"", _lib.DEC_INVALID_BINARY), (bytes([T, 1, 130]) + good[3:], _lib.DEC_MALFORMED),
        (good[:-1], _lib.DEC_MALFORMED), (good + b"\0", _lib.DEC_MALFORMED),
        (good[:len(good) // 2], _lib.DEC_MALFORMED), (bad_flag, _lib.DEC_MALFORMED),
        (unknown, _lib.DEC_UNKNOWN_TERM), (out_of_order, _lib.DEC_UNKNOWN_TERM),
        (no_tokens, _lib.DEC_UNREPRESENTABLE),
        (oetf.to_binary(T, 1, []), _lib.DEC_OK),
        # token count larger / smaller than the records present, count cut short
        (good.replace(bytes([108, 0, 0, 0, 2]), bytes([108, 0, 0, 0, 3]), 1),
         _lib.DEC_UNKNOWN_TERM),
        (good.replace(bytes([108, 0, 0, 0, 2]), bytes([108, 0, 0, 0, 1]), 1),
         _lib.DEC_MALFORMED),
        (good[:good.index(bytes([108, 0, 0, 0, 2])) + 3], _lib.DEC_MALFORMED),
        # a duplicated record (same token twice) is out of term order
        (oetf.to_binary(T, 1, [(1, [(tok[0], False), (tok[0], True)])]),
         _lib.DEC_UNKNOWN_TERM),
        # an unknown token after a bad flag: the flag comes first in stream order
        (oetf.to_binary(T, 1, [(1, [(tok[0], False), (b"z" * 20, True)])])
         .replace(b"false", b"falsx", 1), _lib.DEC_MALFORMED),
    ]
    pay, offs = _upload_payloads(ctx, [c[0] for c in cases])
    b = ctx.orset_batch(len(cases), E)
    with _read_kernel(ctx, knob):
        st = b.etf_decode(d, pay, offs, tag=T, vers=1)
    assert list(st) == [c[1] for c in cases]
    cells = b.download()
    want = dom.encode_orset([s0], E)[0]
    for i in (0, 1, 2):
        assert np.array_equal(cells[i], want)
    assert not cells[14].any()


@pytest.mark.gpu
@pytest.mark.parametrize("knob", [0, 1, 4])
def test_gpu_from_binary_large_round_trip(knob):
    """4096 replicas x 512 slots x 64 token slots: device to_binary then from_binary
    restores every cell."""
    import numpy as np
    from lasp_amd import engine, etf
    from lasp_amd.codec import Domain
    from lasp_amd.orset import context
    from oracle import columnar as orc
    R, E = 4096, 512
    ctx = context()
    b = ctx.orset_batch(R, E)
    b.fill_synthetic(17)
    toks = orc.synth_tokens(E)
    dom = Domain()
    for e in range(E):
        es = dom.element_slot(e)
        for k in range(64):
            dom.token_slot(es, bytes(toks[e][k]))
    d = engine.ETFDict(ctx, E, *dom.etf_arrays(E))
    offs, out, _ = b.etf_encode(d, tag=etf.DT_ORSET_TAG, vers=1)
    b2 = ctx.orset_batch(R, E)
    with _read_kernel(ctx, knob):
        st = b2.etf_decode(d, out, offs, tag=etf.DT_ORSET_TAG, vers=1)
    assert (st == 0).all()
    assert np.array_equal(b2.download(), b.download())


@pytest.mark.gpu
def test_gpu_from_binary_fuzz():
    """2000 corrupted payloads (byte flips, truncations, insertions, splices of two
    payloads): every status is a LASPJ_DEC_* code, a payload that decodes OK re-encodes
    to itself, the batched and the serial decode agree on every status and cell, and
    nothing faults."""
    import numpy as np
    from lasp_amd import etf
    rng = random.Random(77)
    states = _random_orsets(rng, 60, mixed=False)
    ctx, dom, E, d = _decode_setup(states)
    T = etf.DT_ORSET_TAG
    base = [oetf.to_binary(T, 1, s) for s in states]
    blobs = []
    for _ in range(2000 * SOAK):
        b = bytearray(rng.choice(base))
        kind = rng.randrange(4)
        if kind == 0 and b:
            for _ in range(rng.randint(1, 3)):
                b[rng.randrange(len(b))] = rng.randrange(256)
        elif kind == 1 and b:
            del b[rng.randrange(len(b)):]
        elif kind == 2:
            pos = rng.randrange(len(b) + 1)
            b[pos:pos] = bytes(rng.randrange(256) for _ in range(rng.randint(1, 9)))
        else:
            other = rng.choice(base)
            b = b[:rng.randrange(len(b) + 1)] + other[rng.randrange(len(other) + 1):]
        blobs.append(bytes(b))
    pay, offs = _upload_payloads(ctx, blobs)
    bt = ctx.orset_batch(len(blobs), E)
    st = bt.etf_decode(d, pay, offs, tag=T, vers=1)
    assert set(np.unique(st)) <= {0, 1, 2, 3, 4, 5}
    bs = ctx.orset_batch(len(blobs), E)
    with _read_kernel(ctx, 1):
        st_serial = bs.etf_decode(d, pay, offs, tag=T, vers=1)
    assert np.array_equal(st, st_serial), np.nonzero(st != st_serial)[0][:10]
    ok0 = st == 0
    assert np.array_equal(bt.download()[ok0], bs.download()[ok0])
    for knob in (4, 10):                     # segment mode: same statuses and cells
        bg = ctx.orset_batch(len(blobs), E)
        with _read_kernel(ctx, knob):
            st_seg = bg.etf_decode(d, pay, offs, tag=T, vers=1)
        assert np.array_equal(st_seg, st_serial), np.nonzero(st_seg != st_serial)[0][:10]
        assert np.array_equal(bg.download()[ok0], bs.download()[ok0])
    ok = np.nonzero(st == 0)[0]
    if len(ok):
        again = bt.to_binaries(d, tag=T, vers=1)
        for i in ok:
            # what decodes OK re-encodes as term_to_binary of the term binary_to_term
            # reads: the payload itself unless the fuzz rewrote an atom into another
            # valid encoding (ATOM_EXT 100 -> ATOM_UTF8_EXT 118 reads as the same atom,
            # and term_to_binary writes ATOM_EXT again)
            assert again[i] == oetf.to_binary(T, 1, oetf.binary_to_term(blobs[i][2:])), i


def _small_orsets(rng, n):
    """Random orddicts whose elements hold <= 3 of their own 20-byte tokens (the
    dictionary's tok_max <= 8: the decoder's element batches); small and large integer
    elements, an atom, and binaries whose element header is longer than 64 bytes."""
    elems = list(range(0, 300, 3)) + [1 << 40, -7, PAtom("ad"), b"b" * 70, b"c" * 61]
    pool = {i: [bytes(rng.randrange(256) for _ in range(20)) for _ in range(3)]
            for i in range(len(elems))}
    from oracle.otp import lists_sort
    res = []
    for _ in range(n):
        d = {}
        for i in rng.sample(range(len(elems)), rng.randint(0, len(elems))):
            d[elems[i]] = {t: rng.random() < 0.4 for t in rng.sample(pool[i], rng.randint(1, 3))}
        keys = lists_sort(list(d.keys()))
        res.append([(k, [(t, d[k][t]) for t in sorted(d[k])]) for k in keys])
    return res


@pytest.mark.gpu
@pytest.mark.parametrize("knob", [0, 1, 2, 4, 6, "seg512"])
def test_gpu_from_binary_small_tokens_round_trip(knob):
    """Elements with <= 3 token slots (element batches under knob 0): oracle payloads
    with every flag atom form decode to the host encoder's cells, and device to_binary ->
    from_binary is the identity, under every read kernel."""
    import numpy as np
    from lasp_amd import _lib, etf
    rng = random.Random(5)
    states = _small_orsets(rng, 300) + [[]]
    ctx, dom, E, d = _decode_setup(states)
    T = etf.DT_ORSET_TAG
    blobs = []
    for i, s in enumerate(states):
        p = oetf.to_binary(T, 1, s)
        if i % 3 == 1:       # SMALL_ATOM_UTF8_EXT flags
            p = p.replace(bytes([100, 0, 4]) + b"true", bytes([119, 4]) + b"true") \
                 .replace(bytes([100, 0, 5]) + b"false", bytes([119, 5]) + b"false")
        elif i % 3 == 2:     # ATOM_UTF8_EXT `true` beside ATOM_EXT `false`
            p = p.replace(bytes([100, 0, 4]) + b"true", bytes([118, 0, 4]) + b"true")
        blobs.append(p)
    pay, offs = _upload_payloads(ctx, blobs)
    b = ctx.orset_batch(len(states), E)
    want = dom.encode_orset(states, E)
    with _read_kernel(ctx, knob):
        st = b.etf_decode(d, pay, offs, tag=T, vers=1)
        assert (st == _lib.DEC_OK).all(), np.nonzero(st)[0][:10]
        assert np.array_equal(b.download(), want)
        offs2, out2, _ = b.etf_encode(d, tag=T, vers=1)
        b2 = ctx.orset_batch(len(states), E)
        assert (b2.etf_decode(d, out2, offs2, tag=T, vers=1) == 0).all()
        assert np.array_equal(b2.download(), want)


@pytest.mark.gpu
def test_gpu_from_binary_small_tokens_fuzz():
    """3000 corrupted small-token payloads and the 80 intact ones: the element-batch
    decode (knob 0), the record-batch decode (2) and the serial scan (1) give the same
    status and cells for every payload."""
    import numpy as np
    from lasp_amd import etf
    rng = random.Random(91)
    states = _small_orsets(rng, 80)
    ctx, dom, E, d = _decode_setup(states)
    T = etf.DT_ORSET_TAG
    base = [oetf.to_binary(T, 1, s) for s in states]
    blobs = []
    for _ in range(3000):
        b = bytearray(rng.choice(base))
        kind = rng.randrange(5)
        if kind == 0 and b:
            for _ in range(rng.randint(1, 3)):
                b[rng.randrange(len(b))] = rng.randrange(256)
        elif kind == 1 and b:
            del b[rng.randrange(len(b)):]
        elif kind == 2:
            pos = rng.randrange(len(b) + 1)
            b[pos:pos] = bytes(rng.randrange(256) for _ in range(rng.randint(1, 9)))
        elif kind == 3 and len(b) > 8:      # a flag / count / tail byte nudged by one
            pos = rng.randrange(2, len(b))
            b[pos] = (b[pos] + rng.choice([1, 255])) & 0xFF
        else:
            other = rng.choice(base)
            b = b[:rng.randrange(len(b) + 1)] + other[rng.randrange(len(other) + 1):]
        blobs.append(bytes(b))
    blobs += base                             # and the payloads themselves
    pay, offs = _upload_payloads(ctx, blobs)
    res = {}
    for knob in (0, 2, 1):
        bt = ctx.orset_batch(len(blobs), E)
        with _read_kernel(ctx, knob):
            st = bt.etf_decode(d, pay, offs, tag=T, vers=1)
        res[knob] = (st, bt.download())
    st0, c0 = res[0]
    assert set(np.unique(st0)) <= {0, 1, 2, 3, 4, 5}
    assert (st0 == 0).sum() >= len(base)
    for knob in (1, 2):
        st, c = res[knob]
        assert np.array_equal(st0, st), (knob, np.nonzero(st0 != st)[0][:10])
        ok = st0 == 0
        assert np.array_equal(c0[ok], c[ok]), knob


@pytest.mark.gpu
def test_gpu_from_binary_small_tokens_large():
    """8192 replicas x 256 slots x <= 3 tokens (the suite's t3 shape, 10 % of elements
    absent): device to_binary -> from_binary restores every cell; the element-batch and
    record-batch kernels agree."""
    import hashlib
    import numpy as np
    from lasp_amd import engine, etf
    from lasp_amd.codec import Domain
    from lasp_amd.orset import context
    R, E = 8192, 256
    ctx = context()
    rng = np.random.default_rng(3)
    h = np.zeros((R, E, 2), np.uint64)
    present = rng.random((R, E)) < 0.9
    h[:, :, 0] = np.where(present, rng.integers(1, 8, (R, E), dtype=np.uint64), 0)
    h[:, :, 1] = h[:, :, 0] & rng.integers(0, 8, (R, E), dtype=np.uint64)
    b = ctx.orset_batch(R, E)
    b.upload(h)
    dom = Domain()
    for e in range(E):
        es = dom.element_slot(e * 1000)
        for k in range(3):
            dom.token_slot(es, hashlib.blake2b(b"%d:%d" % (e, k), digest_size=20).digest())
    d = engine.ETFDict(ctx, E, *dom.etf_arrays(E))
    offs, out, _ = b.etf_encode(d, tag=etf.DT_ORSET_TAG, vers=1)
    for knob in (0, 2):
        b2 = ctx.orset_batch(R, E)
        with _read_kernel(ctx, knob):
            st = b2.etf_decode(d, out, offs, tag=etf.DT_ORSET_TAG, vers=1)
        assert (st == 0).all(), knob
        assert np.array_equal(b2.download(), h), knob


@pytest.mark.gpu
@pytest.mark.parametrize("knob", [0, 4, 10])
def test_gpu_from_binary_segments(knob):
    """Long payloads split between waves (automatic for a few long payloads, knob 0;
    every payload in 256-byte segments, knob 4): one 10k-element orddict, a few 2k-element
    ones and short ones decode to the host encoder's cells.  Tokens that embed a real
    element header (106 104 2 <elem image> 108) plant false segment starts: those
    replicas fail the chain check and are decoded again serially, with the same result.
    A LIST_EXT of 0 elements with its nil tail is [] (binary_to_term/1 accepts it), one
    without the tail is malformed."""
    import numpy as np
    from lasp_amd import _lib, etf
    rng = random.Random(11)
    trap = lambda e, k: bytes([106, 104, 2, 97, e, 108]) + bytes([k]) * 14   # noqa: E731
    big = [(e, [(bytes([e % 251, k]) * 10, rng.random() < 0.5) for k in range(2)])
           for e in range(10_000)]
    mids = [[(e, sorted([(trap((e + 7) % 200, k) if e % 5 == 0 else
                          bytes([k, e % 256]) * 10, rng.random() < 0.3) for k in range(3)]))
             for e in range(i, 2000 + i)] for i in range(3)]
    states = [big] + mids + [[], [(1, [(bytes([1, 1]) * 10, True)])]]
    ctx, dom, E, d = _decode_setup(states)
    T = etf.DT_ORSET_TAG
    blobs = [oetf.to_binary(T, 1, s) for s in states]
    blobs += [bytes([T, 1, 131, 108, 0, 0, 0, 0, 106]), bytes([T, 1, 131, 108, 0, 0, 0, 0])]
    pay, offs = _upload_payloads(ctx, blobs)
    b = ctx.orset_batch(len(blobs), E)
    with _read_kernel(ctx, knob):
        st = b.etf_decode(d, pay, offs, tag=T, vers=1)
    assert list(st) == [_lib.DEC_OK] * (len(states) + 1) + [_lib.DEC_MALFORMED]
    want = dom.encode_orset(states + [[]], E)
    assert np.array_equal(b.download()[:len(states) + 1], want)
    assert etf.binary_to_term(bytes([131, 108, 0, 0, 0, 0, 106])) == []


@pytest.mark.gpu
def test_gpu_from_binary_record_locator_fuzz():
    """Elements with 20-40 records (the byte-parallel record locator's case), tokens that
    embed its `101 104 2` marker at every offset, flags in all three atom forms, and
    1500 corrupted copies: the batched decode (locator + chain fallback) and the serial
    scan agree on every status and cell, and clean payloads decode to the encoder's
    cells."""
    import numpy as np
    from lasp_amd import etf
    rng = random.Random(404)
    marker = bytes([101, 104, 2])

    def tok(i, k):
        b = bytearray(rng.randrange(256) for _ in range(20))
        if k % 3 == 0:
            at = (i + k) % 18
            b[at:at + 3] = marker
        return bytes(b)
    pools = {e: sorted({tok(e, k) for k in range(48)}) for e in range(40)}
    states = []
    for _ in range(30):
        es = sorted(rng.sample(range(40), rng.randint(1, 12)))
        states.append([(e, sorted((t, rng.random() < 0.5)
                                  for t in rng.sample(pools[e], rng.randint(20, 40))))
                       for e in es])
    ctx, dom, E, d = _decode_setup(states)
    T = etf.DT_ORSET_TAG
    base = []
    for i, s in enumerate(states):
        p = oetf.to_binary(T, 1, s)
        if i % 3 == 1:
            p = p.replace(bytes([100, 0, 4]) + b"true", bytes([119, 4]) + b"true") \
                 .replace(bytes([100, 0, 5]) + b"false", bytes([119, 5]) + b"false")
        elif i % 3 == 2:
            p = p.replace(bytes([100, 0, 5]) + b"false", bytes([118, 0, 5]) + b"false")
        base.append(p)
    blobs = list(base)
    for _ in range(1500):
        b = bytearray(rng.choice(base))
        kind = rng.randrange(4)
        if kind == 0:
            for _ in range(rng.randint(1, 2)):
                b[rng.randrange(len(b))] = rng.choice([101, 104, 2, 106, 5, 4, rng.randrange(256)])
        elif kind == 1:
            del b[rng.randrange(len(b)):]
        elif kind == 2:
            pos = rng.randrange(len(b) + 1)
            b[pos:pos] = rng.choice([marker, bytes([101]), bytes([104, 2]), b"\0"])
        else:
            pos = rng.randrange(len(b))
            del b[pos:pos + rng.randint(1, 3)]
        blobs.append(bytes(b))
    pay, offs = _upload_payloads(ctx, blobs)
    bt = ctx.orset_batch(len(blobs), E)
    st = bt.etf_decode(d, pay, offs, tag=T, vers=1)
    bs = ctx.orset_batch(len(blobs), E)
    with _read_kernel(ctx, 1):
        st_serial = bs.etf_decode(d, pay, offs, tag=T, vers=1)
    assert np.array_equal(st, st_serial), np.nonzero(st != st_serial)[0][:10]
    ok = st == 0
    assert np.array_equal(bt.download()[ok], bs.download()[ok])
    assert (st[:len(base)] == 0).all()
    assert np.array_equal(bt.download()[:len(base)], dom.encode_orset(states, E))


@pytest.mark.gpu
@pytest.mark.parametrize("seed", [4242 + i for i in range(SOAK)])
def test_gpu_from_binary_many_token_batches_fuzz(seed):
    """Many-token dictionaries (up to 64 token slots per element), elements of 1 to 64
    records, so a batch holds one to several whole elements or stops inside one; tokens
    that embed the batch's item marker 104 2 and whole false element starts (106 104 2
    <a real element header>), flags in all three atom forms, and 2500 corrupted copies:
    element batches (knob 0), one element at a time (7) and the
    serial scan (1) agree on every status and cell, and the clean payloads decode to the
    encoder's cells."""
    import numpy as np
    from lasp_amd import etf
    rng = random.Random(seed)
    T = etf.DT_ORSET_TAG
    elems = list(range(0, 120, 2)) + [300, 1 << 33]

    def hdr(x):
        return bytes(oetf.term_to_binary([(x, [(b"", False)])])[6:])[:2 + (2 if x < 256 else 5)]

    def tok(i, k):
        b = bytearray(rng.randrange(256) for _ in range(20))
        kind = k % 5
        if kind == 0:
            at = (i + k) % 19
            b[at:at + 2] = bytes([104, 2])
        elif kind == 1:
            h = bytes([106]) + hdr(elems[(i + k) % len(elems)]) + bytes([108])
            at = (i * 7 + k) % (21 - len(h))
            b[at:at + len(h)] = h
        return bytes(b)
    pools = {e: sorted({tok(i, k) for k in range(64)}) for i, e in enumerate(elems)}
    states = []
    for n in range(60):
        es = sorted(rng.sample(elems, rng.randint(1, 14)))
        sizes = [1, 2, 5, 20, 33, 63, 64]
        states.append([(e, sorted((t, rng.random() < 0.5) for t in
                                  rng.sample(pools[e], rng.choice(sizes)))) for e in es])
    ctx, dom, E, d = _decode_setup(states)
    base = []
    for i, s in enumerate(states):
        p = oetf.to_binary(T, 1, s)
        if i % 3 == 1:
            p = p.replace(bytes([100, 0, 4]) + b"true", bytes([119, 4]) + b"true") \
                 .replace(bytes([100, 0, 5]) + b"false", bytes([119, 5]) + b"false")
        elif i % 3 == 2:
            p = p.replace(bytes([100, 0, 5]) + b"false", bytes([118, 0, 5]) + b"false")
        base.append(p)
    blobs = list(base)
    for _ in range(2500):
        b = bytearray(rng.choice(base))
        kind = rng.randrange(5)
        if kind == 0:
            for _ in range(rng.randint(1, 2)):
                b[rng.randrange(len(b))] = rng.choice([101, 104, 2, 106, 108, 0, 5, 4,
                                                       rng.randrange(256)])
        elif kind == 1:
            del b[rng.randrange(len(b)):]
        elif kind == 2:
            pos = rng.randrange(len(b) + 1)
            b[pos:pos] = rng.choice([bytes([104, 2]), bytes([106, 104, 2]), bytes([106]),
                                     b"\0"])
        elif kind == 3:
            pos = rng.randrange(len(b))
            del b[pos:pos + rng.randint(1, 3)]
        else:                                  # an element's count nudged by one
            at = [i for i in range(len(b) - 4) if b[i] == 108 and b[i + 1:i + 3] == b"\0\0"]
            if at:
                i = rng.choice(at) + 4
                b[i] = (b[i] + rng.choice([1, 255])) & 0xFF
        blobs.append(bytes(b))
    pay, offs = _upload_payloads(ctx, blobs)
    res = {}
    for knob in (0, 7, 1):
        bt = ctx.orset_batch(len(blobs), E)
        with _read_kernel(ctx, knob):
            st = bt.etf_decode(d, pay, offs, tag=T, vers=1)
        res[knob] = (st, bt.download())
    st0, c0 = res[0]
    assert set(np.unique(st0)) <= {0, 1, 2, 3, 4, 5}
    assert (st0[:len(base)] == 0).all(), np.nonzero(st0[:len(base)])[0][:10]
    assert np.array_equal(c0[:len(base)], dom.encode_orset(states, E))
    for knob in (7, 1):
        st, c = res[knob]
        assert np.array_equal(st0, st), (knob, np.nonzero(st0 != st)[0][:10])
        ok = st0 == 0
        assert np.array_equal(c0[ok], c[ok]), knob


@pytest.mark.gpu
def test_gpu_from_binary_small_tokens_fuzz():
    """Elements with <= 3 token slots (the lane-parallel element batches): tokens that
    embed the element-start marker `106 104 2` followed by a real element header, and
    1500 corrupted payloads; the default decode, the scalar-walk element batches (knob 6)
    and the serial scan agree on every status and cell."""
    import numpy as np
    from lasp_amd import etf
    rng = random.Random(606)
    states = _small_orsets(rng, 200)
    hdrs = [bytes([106, 104, 2, 97, x, 108]) for x in range(0, 60, 3)]
    memo = {}

    def plant(t):
        # the same rewrite every time a token appears: elements keep their <= 3 tokens
        if t not in memo:
            h = rng.choice(hdrs)
            at = rng.randrange(0, 20 - len(h) + 1)
            memo[t] = t[:at] + h + t[at + len(h):] if rng.random() < 0.4 else t
        return memo[t]
    planted = [[(e, sorted(dict((plant(t), f) for t, f in toks).items())) for e, toks in s_]
               for s_ in states]
    ctx, dom, E, d = _decode_setup(planted)
    T = etf.DT_ORSET_TAG
    base = [oetf.to_binary(T, 1, s_) for s_ in planted]
    blobs = list(base)
    for _ in range(1500):
        b = bytearray(rng.choice(base))
        kind = rng.randrange(4)
        if kind == 0 and b:
            for _ in range(rng.randint(1, 2)):
                b[rng.randrange(len(b))] = rng.choice([106, 104, 2, 108, 97, rng.randrange(256)])
        elif kind == 1 and b:
            del b[rng.randrange(len(b)):]
        elif kind == 2:
            pos = rng.randrange(len(b) + 1)
            b[pos:pos] = rng.choice([bytes([106, 104, 2]), bytes([106]), b"\0"])
        elif b:
            pos = rng.randrange(len(b))
            del b[pos:pos + rng.randint(1, 3)]
        blobs.append(bytes(b))
    pay, offs = _upload_payloads(ctx, blobs)
    res = {}
    for knob in (0, 6, 1):
        bt = ctx.orset_batch(len(blobs), E)
        with _read_kernel(ctx, knob):
            st = bt.etf_decode(d, pay, offs, tag=T, vers=1)
        res[knob] = (st, bt.download())
    st1, c1 = res[1]
    for knob in (0, 6):
        st, cl = res[knob]
        assert np.array_equal(st, st1), (knob, np.nonzero(st != st1)[0][:10])
        ok = st1 == 0
        assert np.array_equal(cl[ok], c1[ok]), knob
    assert (st1[:len(base)] == 0).all()
    assert np.array_equal(res[0][1][:len(base)], dom.encode_orset(planted, E))


# ------------------------------------------------------------------ G-Set from_binary

def _random_gsets(rng, n):
    from oracle.otp import lists_usort
    pool = ([0, 1, 7, 255, 256, 1000, -3, 1 << 40, -(1 << 70), 2.5] +
            [PAtom(a) for a in ("a", "b", "zz")] + [(1, 2), (PAtom("k"), b"v")] +
            [bytes(rng.randrange(256) for _ in range(rng.randint(0, 30))) for _ in range(20)] +
            list(range(300, 340)))
    out = [[], [0, 1, 255], list(range(0, 256, 3)), list(range(300)), [PAtom("a"), (1, 2), b"x"]]
    for _ in range(n):
        out.append(lists_usort(rng.sample(pool, rng.randint(0, len(pool)))))
    return out


def _gset_decode_setup(states):
    from lasp_amd import engine
    from lasp_amd.codec import Domain
    from lasp_amd.orset import context
    dom = Domain()
    dom.encode_gset(states, 1 << 12)
    E = dom.size + 3
    ctx = context()
    return ctx, dom, E, engine.ETFDict(ctx, E, *dom.etf_arrays(E, tokens=False))


@pytest.mark.gpu
@pytest.mark.parametrize("knob", [0, 6, 1])
def test_gpu_gset_to_binary_few_long_payloads(knob):
    """Few long G-Set payloads (the NIF's value/1 and merge answers): the split writer
    (chunks of 256 term-order slots over the chip, LASPJ_TUNE_ETF_KERNEL 0), the one-wave
    writer (6) and the block writer (1) give the oracle's term_to_binary byte for byte:
    10k integers (2- and 5-byte images), every byte integer (STRING_EXT), [], mixed terms
    (atoms, binaries, tuples, big and negative integers), a set whose elements sit in the
    last chunk only; the public size / write pair and bare / tagged payloads; a present slot
    without an image, or a bit past the dictionary, is refused."""
    import numpy as np
    from lasp_amd import _lib, etf
    from lasp_amd.codec import Domain
    from lasp_amd.orset import context
    from lasp_amd import engine
    from oracle.otp import lists_usort
    rng = random.Random(29)
    mixed = lists_usort([rng.randrange(-500, 70000) for _ in range(900)] +
                        [PAtom("k" * rng.randint(1, 30)) for _ in range(40)] +
                        [bytes(rng.randrange(256) for _ in range(rng.randint(0, 40)))
                         for _ in range(60)] + [(rng.randrange(5), PAtom("t")) for _ in range(9)] +
                        [1 << 40, -(1 << 35)])
    states = [list(range(0, 30000, 3)), list(range(256)), [], mixed, list(range(29990, 30000))]
    dom = Domain(element_capacity=1 << 16)
    dom.encode_gset(states, 1 << 16)
    E = dom.size + 5
    ctx = context()
    d = engine.ETFDict(ctx, E, *dom.etf_arrays(E, tokens=False))
    b = ctx.gset_batch(len(states), E)
    b.upload(dom.encode_gset(states, E))
    ctx.set_tuning(_lib.TUNE_ETF_KERNEL, knob)
    try:
        for tag in (-1, etf.DT_GSET_TAG):
            got = b.to_binaries(d, tag=tag, vers=1)
            for st, g in zip(states, got):
                want = oetf.to_binary(tag, 1, st) if tag >= 0 else oetf.term_to_binary(st)
                assert g == want, (len(st), len(g), len(want))
        words = dom.encode_gset(states, E)
        words[1, (E - 2) >> 6] |= np.uint64(1) << np.uint64((E - 2) & 63)    # no image
        b.upload(words)
        with pytest.raises(_lib.LaspjError):
            b.etf_encode(d)
        if E & 63:
            words = dom.encode_gset(states, E)
            words[3, E >> 6] |= np.uint64(1) << np.uint64(63)                  # past E
            b.upload(words)
            with pytest.raises(_lib.LaspjError):
                b.etf_encode(d)
    finally:
        ctx.set_tuning(_lib.TUNE_ETF_KERNEL, 0)


@pytest.mark.gpu
@pytest.mark.parametrize("tagged", [False, True])
def test_gpu_gset_from_binary_round_trip(tagged):
    """lasp_gset:from_binary/1 on the device (laspj_gset_etf_read): term_to_binary
    payloads of random ordsets — STRING_EXT (every element 0..255), LIST_EXT of mixed
    terms, [] — give the host encoder's words, and device to_binary -> from_binary is the
    identity."""
    import numpy as np
    from lasp_amd import _lib, etf
    states = _random_gsets(random.Random(5 + tagged), 150)
    ctx, dom, E, d = _gset_decode_setup(states)
    tag = etf.DT_GSET_TAG if tagged else -1
    blobs = [oetf.to_binary(tag, 1, s) if tagged else oetf.term_to_binary(s) for s in states]
    assert blobs[2][2 if tagged else 0:][:2] == bytes([131, 107])      # a STRING_EXT case
    pay, offs = _upload_payloads(ctx, blobs)
    b = ctx.gset_batch(len(states), E)
    st = b.etf_decode(d, pay, offs, tag=tag, vers=1)
    assert (st == _lib.DEC_OK).all(), np.nonzero(st)[0][:10]
    want = dom.encode_gset(states, E)
    assert np.array_equal(b.download(), want)
    offs2, out2, _ = b.etf_encode(d, tag=tag, vers=1)
    b2 = ctx.gset_batch(len(states), E)
    assert (b2.etf_decode(d, out2, offs2, tag=tag, vers=1) == 0).all()
    assert np.array_equal(b2.download(), want)


@pytest.mark.gpu
def test_gpu_gset_from_binary_errors():
    """Statuses as the OR-Set decoder's: ?INVALID_BINARY, ?UNSUPPORTED_VERSION, malformed
    (no 131, truncated, trailing byte, improper tail, not a list), elements outside the
    dictionary, not strictly ascending (out of order, repeated, 1 next to 1.0), and
    terms no dictionary holds (a pid)."""
    from lasp_amd import _lib, etf
    T = etf.DT_GSET_TAG
    s0 = [1, 5, PAtom("a"), b"xy"]
    # (the dictionary holds 1, not 1.0: a Domain refuses a second term of one `==` class)
    ctx, dom, E, d = _gset_decode_setup([s0, [2, 300]])
    good = oetf.to_binary(T, 1, s0)
    improper = good[:-1] + bytes([97, 3])                 # [1, 5, a, <<"xy">> | 3]
    pid = bytes([T, 1, 131, 108, 0, 0, 0, 1, 88]) + bytes([100, 0, 1]) + b"n" + bytes(12) + bytes([106])
    cases = [
        (good, _lib.DEC_OK),
        (oetf.to_binary(T, 1, []), _lib.DEC_OK),
        (oetf.to_binary(T, 1, [2]), _lib.DEC_OK),                      # STRING_EXT [2]
        (oetf.to_binary(T, 1, [1, 2, 5]), _lib.DEC_OK),
        (bytes([T + 1]) + good[1:], _lib.DEC_INVALID_BINARY),
        (b"", _lib.DEC_INVALID_BINARY),
        (bytes([T, 2]) + good[2:], _lib.DEC_UNSUPPORTED_VERSION),
        (bytes([T, 1, 130]) + good[3:], _lib.DEC_MALFORMED),
        (good[:-1], _lib.DEC_MALFORMED), (good + b"\0", _lib.DEC_MALFORMED),
        (good[:len(good) // 2], _lib.DEC_MALFORMED), (improper, _lib.DEC_MALFORMED),
        (oetf.to_binary(T, 1, PAtom("a")), _lib.DEC_MALFORMED),         # not a list
        (oetf.to_binary(T, 1, [7]), _lib.DEC_UNKNOWN_TERM),             # not in the dictionary
        (oetf.to_binary(T, 1, [PAtom("zz")]), _lib.DEC_UNKNOWN_TERM),
        (oetf.to_binary(T, 1, [5, 1]), _lib.DEC_UNKNOWN_TERM),          # out of order
        (oetf.to_binary(T, 1, [1, 1]), _lib.DEC_UNKNOWN_TERM),          # repeated
        (oetf.to_binary(T, 1, [1, 1.0]), _lib.DEC_UNKNOWN_TERM),        # 1 == 1.0
        (oetf.to_binary(T, 1, [2, 2]), _lib.DEC_UNKNOWN_TERM),          # STRING_EXT repeated
        (pid, _lib.DEC_UNKNOWN_TERM),                                   # a pid: binary_to_term
    ]
    pay, offs = _upload_payloads(ctx, [c[0] for c in cases])
    b = ctx.gset_batch(len(cases), E)
    st = b.etf_decode(d, pay, offs, tag=T, vers=1)
    assert list(st) == [c[1] for c in cases]
    assert list(b.download()[0]) == list(dom.encode_gset([s0], E)[0])


@pytest.mark.gpu
@pytest.mark.parametrize("knob", [0, 11, 12, 13, 14])
def test_gpu_gset_from_binary_long_payloads(knob):
    """Payloads longer than the decoder's 4 KiB window (the walk restages it): 10k
    integers (2- and 5-byte images: runs of equal lengths taken 64 at a time), mixed
    terms with atoms, binaries and tuples of many lengths, a binary longer than the
    window, and elements straddling window edges; then the same payloads truncated at
    and around window edges, with a trailing byte, an improper tail, an element outside
    the dictionary, and two elements swapped deep inside — each with its status."""
    import numpy as np
    from lasp_amd import _lib, engine, etf
    from lasp_amd.codec import Domain
    from lasp_amd.orset import context
    from oracle.otp import lists_usort
    rng = random.Random(17)
    T = etf.DT_GSET_TAG
    mixed = lists_usort([rng.randrange(70000) for _ in range(1500)] +
                        [PAtom("a" * rng.randint(1, 40)) for _ in range(60)] +
                        [bytes(rng.randrange(256) for _ in range(rng.randint(0, 100)))
                         for _ in range(200)] +
                        [(rng.randrange(9), b"t" * rng.randrange(30)) for _ in range(50)] +
                        [b"L" * 6000])
    states = [list(range(0, 70000, 7)), mixed, list(range(300)), list(range(256, 2256)),
              lists_usort([b"x" * k for k in range(0, 300, 3)])]
    dom = Domain(element_capacity=1 << 16)
    dom.encode_gset(states, 1 << 16)
    E = dom.size + 5
    ctx = context()
    d = engine.ETFDict(ctx, E, *dom.etf_arrays(E, tokens=False))
    good = [oetf.to_binary(T, 1, s) for s in states]
    assert all(len(g) > 4096 for g in good[:2])
    cases = [(g, _lib.DEC_OK) for g in good]
    L0 = good[0]
    for cut in (4096, 4097, 4100, 8190, 8192, len(L0) - 1, len(L0) // 2 + 1):
        cases.append((L0[:cut], _lib.DEC_MALFORMED))
    cases.append((good[1][:4096 + 13], _lib.DEC_MALFORMED))
    cases.append((L0 + b"\0", _lib.DEC_MALFORMED))
    cases.append((L0[:-1] + bytes([97, 3]), _lib.DEC_MALFORMED))           # improper tail
    # element 5000 of range(0, 70000, 7) is 35000 (INTEGER_EXT): make it 99999 (in no set)
    i5000 = L0.index(bytes([98]) + (35000).to_bytes(4, "big"))
    cases.append((L0[:i5000 + 1] + (99999).to_bytes(4, "big") + L0[i5000 + 5:],
                  _lib.DEC_UNKNOWN_TERM))
    j = L0.index(bytes([98]) + (49000).to_bytes(4, "big"))                # swap two
    swapped = L0[:j] + L0[j + 5:j + 10] + L0[j:j + 5] + L0[j + 10:]
    cases.append((swapped, _lib.DEC_UNKNOWN_TERM))
    pay, offs = _upload_payloads(ctx, [c[0] for c in cases])
    b = ctx.gset_batch(len(cases), E)
    with _read_kernel(ctx, knob):
        st = b.etf_decode(d, pay, offs, tag=T, vers=1)
    assert list(st) == [c[1] for c in cases]
    assert np.array_equal(b.download()[:len(states)], dom.encode_gset(states, E))


@pytest.mark.gpu
def test_gpu_gset_from_binary_split_fuzz():
    """The split decoder of few long payloads (element extents by one wave per payload,
    the elements resolved over the chip; LASPJ_TUNE_ETF_READ 0) against the one-wave
    decoder (15, which the oracle fuzz above pins): 6 x 120 long payloads (integers of
    2- and 5-byte images, mixed terms, every byte integer) intact and corrupted (bytes
    changed, truncated, bytes inserted, two payloads spliced, two elements swapped) give
    the same statuses, and the same words where OK."""
    import numpy as np
    from lasp_amd import _lib, engine, etf
    from lasp_amd.codec import Domain
    from lasp_amd.orset import context
    from oracle.otp import lists_usort
    rng = random.Random(53)
    T = etf.DT_GSET_TAG
    mixed = lists_usort([rng.randrange(-300, 90000) for _ in range(1500)] +
                        [PAtom("m" * rng.randint(1, 20)) for _ in range(30)] +
                        [bytes(rng.randrange(256) for _ in range(rng.randint(0, 30)))
                         for _ in range(40)] + [(rng.randrange(4), PAtom("u")) for _ in range(6)])
    pool = [list(range(0, 40000, 3)), mixed, list(range(256, 3000)), list(range(0, 90000, 7))]
    dom = Domain(element_capacity=1 << 17)
    dom.encode_gset(pool + [list(range(256))], 1 << 17)
    E = dom.size + 3
    ctx = context()
    d = engine.ETFDict(ctx, E, *dom.etf_arrays(E, tokens=False))
    for rnd in range(6 * SOAK):
        base = []
        for _ in range(8):
            src = rng.choice(pool)
            base.append(oetf.to_binary(T, 1, lists_usort(rng.sample(src, rng.randint(len(src) // 2, len(src))))))
        base.append(oetf.to_binary(T, 1, list(range(256))))
        blobs = list(base)
        while len(blobs) < 120:
            b = bytearray(rng.choice(base))
            kind = rng.randrange(5)
            if kind == 0:
                for _ in range(rng.randint(1, 3)):
                    b[rng.randrange(2, len(b))] = rng.randrange(256)
            elif kind == 1:
                del b[rng.randrange(2, len(b) + 1):]
            elif kind == 2:
                pos = rng.randrange(2, len(b) + 1)
                b[pos:pos] = bytes(rng.randrange(256) for _ in range(rng.randint(1, 9)))
            elif kind == 3:
                other = rng.choice(base)
                b = b[:rng.randrange(2, len(b) + 1)] + other[rng.randrange(2, len(other) + 1):]
            else:
                j = rng.randrange(7, max(8, len(b) - 12))
                if b[j] == 98 and b[j + 5] == 98:
                    b[j:j + 10] = b[j + 5:j + 10] + b[j:j + 5]
            blobs.append(bytes(b))
        pay, offs = _upload_payloads(ctx, blobs)
        got = {}
        for knob in (0, 15):
            bt = ctx.gset_batch(len(blobs), E)
            with _read_kernel(ctx, knob):
                st = bt.etf_decode(d, pay, offs, tag=T, vers=1)
            got[knob] = (st, bt.download())
        assert list(got[0][0]) == list(got[15][0]), rnd
        ok = got[0][0] == _lib.DEC_OK
        assert ok[:len(base)].all()
        assert np.array_equal(got[0][1][ok], got[15][1][ok]), rnd


@pytest.mark.gpu
@pytest.mark.parametrize("tagged", [False, True])
def test_gpu_gset_from_binary_split_edges(tagged):
    """The split decoder's edges against the one-wave decoder and the host encoder: a batch
    of few payloads mixing long ones (just past the 4 KiB split threshold, and 30k
    elements: a walk over several 32 KiB windows) with [], one element, every byte integer
    (STRING_EXT) and an empty payload; bare and tagged."""
    import numpy as np
    from lasp_amd import _lib, engine, etf
    from lasp_amd.codec import Domain
    from lasp_amd.orset import context
    T = etf.DT_GSET_TAG if tagged else -1
    long_ = list(range(0, 90000, 3))
    states = [long_, [], [7], list(range(256)), list(range(300, 300 + 820)), long_[::2], []]
    dom = Domain(element_capacity=1 << 17)
    dom.encode_gset(states, 1 << 17)
    E = dom.size + 3
    ctx = context()
    d = engine.ETFDict(ctx, E, *dom.etf_arrays(E, tokens=False))
    enc = lambda st: oetf.to_binary(T, 1, st) if tagged else oetf.term_to_binary(st)  # noqa: E731
    blobs = [enc(st) for st in states[:-1]] + [b""]
    assert len(blobs[4]) > 4096 and len(blobs[0]) > 4 * 32768
    pay, offs = _upload_payloads(ctx, blobs)
    got = {}
    for knob in (0, 15):
        bt = ctx.gset_batch(len(blobs), E)
        with _read_kernel(ctx, knob):
            st = bt.etf_decode(d, pay, offs, tag=T, vers=1)
        got[knob] = (list(st), bt.download())
    assert got[0][0] == got[15][0]
    want_st = [_lib.DEC_OK] * (len(blobs) - 1) + [_lib.DEC_INVALID_BINARY if tagged
                                                  else _lib.DEC_MALFORMED]
    assert got[0][0] == want_st
    want = dom.encode_gset(states, E)
    assert np.array_equal(got[0][1][:-1], want[:-1])
    assert np.array_equal(got[15][1][:-1], want[:-1])


@pytest.mark.gpu
@pytest.mark.parametrize("knob", [0, 11, 13])
def test_gpu_gset_from_binary_fuzz(knob):
    """2000 corrupted G-Set payloads against the oracle's binary_to_term: payloads it
    decodes to an ordset of dictionary terms decode OK to the host encoder's words; other
    lists give UNKNOWN_TERM, non-lists and structural failures MALFORMED (a tag the oracle
    decoder lacks may also read as UNKNOWN_TERM, which the NIF hands to binary_to_term);
    nothing faults."""
    import numpy as np
    from lasp_amd import _lib, etf
    from oracle.otp import lists_usort
    from oracle.terms import exact_eq as eq
    rng = random.Random(91)
    states = _random_gsets(rng, 60)
    ctx, dom, E, d = _gset_decode_setup(states)
    T = etf.DT_GSET_TAG
    base = [oetf.to_binary(T, 1, s) for s in states]
    blobs = list(base)                     # the intact payloads decode too
    for _ in range(2000 * SOAK):
        b = bytearray(rng.choice(base))
        kind = rng.randrange(4)
        if kind == 0 and len(b) > 2:
            for _ in range(rng.randint(1, 3)):
                b[rng.randrange(2, len(b))] = rng.randrange(256)
        elif kind == 1:
            del b[rng.randrange(2, len(b) + 1):]
        elif kind == 2:
            pos = rng.randrange(2, len(b) + 1)
            b[pos:pos] = bytes(rng.randrange(256) for _ in range(rng.randint(1, 9)))
        else:
            other = rng.choice(base)
            b = b[:rng.randrange(2, len(b) + 1)] + other[rng.randrange(2, len(other) + 1):]
        blobs.append(bytes(b))
    pay, offs = _upload_payloads(ctx, blobs)
    bt = ctx.gset_batch(len(blobs), E)
    with _read_kernel(ctx, knob):
        st = bt.etf_decode(d, pay, offs, tag=T, vers=1)
    words = bt.download()
    eb, eo, _o, *_ = dom.etf_arrays(E, tokens=False)
    images = {bytes(eb[eo[k]:eo[k + 1]]): k for k in range(dom.size)}

    def raw_elements(b):
        """the element images as they stand in a well-formed list payload"""
        if b[1] == 106:
            return []
        if b[1] == 107:
            n = int.from_bytes(b[2:4], "big")
            return [bytes([97, v]) for v in b[4:4 + n]]
        n, i, out = int.from_bytes(b[2:6], "big"), 6, []
        for _ in range(n):
            j = oetf._dec(b, i)[1]
            out.append(bytes(b[i:j]))
            i = j
        return out
    n_ok = 0
    for i, blob in enumerate(blobs):
        try:
            term = oetf.binary_to_term(blob[2:])
            why = None
        except Exception as e:            # binary_to_term raises badarg
            term, why = None, str(e)
        if term is None:
            lax = "external tag" in why or (len(blob) > 3 and blob[3] == 80)
            assert st[i] in ((_lib.DEC_MALFORMED, _lib.DEC_UNKNOWN_TERM) if lax
                             else (_lib.DEC_MALFORMED,)), (i, why, st[i])
            continue
        if not isinstance(term, list):
            assert st[i] == _lib.DEC_MALFORMED, i
            continue
        is_set = eq(lists_usort(term), term) and all(r in images for r in raw_elements(blob[2:]))
        if not is_set:
            assert st[i] == _lib.DEC_UNKNOWN_TERM, (i, term)
            continue
        assert st[i] == _lib.DEC_OK, (i, term)
        n_ok += 1
        want = np.zeros_like(words[i])
        for r in raw_elements(blob[2:]):
            k = images[r]
            want[k >> 6] |= np.uint64(1 << (k & 63))
        assert np.array_equal(words[i], want), i
    assert n_ok >= len(base)
