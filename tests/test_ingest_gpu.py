"""GPU parity of the CR ingest (kdtn_json_ingest, kdtn_ingest.hip) against the C oracle's
decode of the same TopologyList documents (oracle/kdtn_oracle_json.c, itself pinned by
tests/test_ingest_cpu.py): every table bit for bit (dictionaries in first-occurrence
order, topology columns and offsets, both link stores), the rejection class of malformed
documents, and JSON → ingest → epoch → batches against the oracle chain.
"""
from __future__ import annotations

import random

import numpy as np
import pytest

import json_ref as jr
import oracle as O
from kdtn import abi, synth
from kdtn.engine import KdtnError
from test_ingest_cpu import (BAD_SYNTAX, GO_ESCAPE_OFFSETS, SEP_SYNTAX, DUPS, GO_STRINGS, TYPE_ERRORS, GOLDEN, rand_topos, s0p,
                             sample_doc)

pytestmark = pytest.mark.gpu
TICK = 15.625


def tables_equal(a, b, ctx=""):
    """EpochInput equality, array by array"""
    pairs = [("kdict.bytes", a.kdict.bytes_, b.kdict.bytes_), ("kdict.offs", a.kdict.offs, b.kdict.offs),
             ("pdict.bytes", a.pdict.bytes_, b.pdict.bytes_), ("pdict.offs", a.pdict.offs, b.pdict.offs)]
    for f in ("ns", "name", "src_ip", "net_ns", "flags", "real_off", "des_off"):
        pairs.append(("topos." + f, getattr(a.topos, f), getattr(b.topos, f)))
    for side in ("desired", "realised"):
        for f in ("key", "prop", "gap", "uid"):
            pairs.append((f"{side}.{f}", getattr(getattr(a, side), f), getattr(getattr(b, side), f)))
    for name, x, y in pairs:
        x, y = np.asarray(x), np.asarray(y)
        if x.shape != y.shape or x.tobytes() != y.tobytes():
            raise AssertionError(f"{ctx}: {name} differs: shape {x.shape} vs {y.shape}; "
                                 f"{x.ravel()[:8]} vs {y.ravel()[:8]}")


def gpu_ingest(engine, doc):
    """(json_err, tables | None) from the GPU"""
    try:
        engine.ingest(doc)
    except KdtnError as e:
        if e.code != abi.EBADMSG:
            raise
        return e.info.json_err, None
    return 0, engine.ingest_tables()


def check_doc(engine, doc, ctx=""):
    e0, _, want = O.json_ingest(doc)
    e1, got = gpu_ingest(engine, doc)
    assert e1 == e0, f"{ctx}: GPU json_err {e1}, oracle {e0}"
    if want is not None:
        tables_equal(got, want, ctx)
    return want


@pytest.mark.parametrize("seed", range(16))
def test_random_documents(engine, seed):
    rng = random.Random(seed)
    root = jr.topology_list(rand_topos(rng, 60 + 20 * seed), rng)
    doc = jr.dumps(root, rng, ws=0.3 if seed % 2 else 0.0, esc=0.08 if seed % 3 == 0 else 0.0).encode()
    check_doc(engine, doc, f"seed {seed}")


@pytest.mark.parametrize("doc", BAD_SYNTAX + TYPE_ERRORS + DUPS)
def test_rejections(engine, doc):
    check_doc(engine, doc, repr(doc[:60]))


def test_separator_error_offsets(engine):
    """Misplaced / repeated / trailing ',' and ':' (the GPU token stream has no separator tokens:
    each token records the separator before it, k_js_tail checks the ones after the last token):
    the rejection lands on the byte the oracle's checkValid stops at, the document's end for a
    truncated one."""
    bad = []
    for doc in SEP_SYNTAX:
        if not doc.strip(b" ,:"):
            continue                                # no token at all: offset 0 by the host check
        e0, off0, _ = O.json_ingest(doc)
        try:
            engine.ingest(doc)
            bad.append((doc, "accepted"))
            continue
        except KdtnError as e:
            if e.code != abi.EBADMSG:
                raise
            e1, off1 = e.info.json_err, e.info.err_offset
        if (e1, off1) != (e0, off0):
            bad.append((doc, (e1, off1), (e0, off0)))
    assert not bad, bad


@pytest.mark.parametrize("doc,go_off", GO_ESCAPE_OFFSETS)
def test_escape_error_offsets(engine, doc, go_off):
    """A bad escape (checked per escaped byte from k_js_quotes' escaped-byte mask, in
    k_js_classify) is rejected where Go's scanner stops: at the escape byte, or at the first
    non-hex digit of \\uXXXX (go_off: the offending byte's index = SyntaxError.Offset - 1; the
    document's length for an escape cut by its end), as the oracle reports it."""
    e0, off0, _ = O.json_ingest(doc)
    assert (e0, off0) == (abi.JSON_SYNTAX, go_off)
    with pytest.raises(KdtnError) as ei:
        engine.ingest(doc)
    assert ei.value.code == abi.EBADMSG
    assert (ei.value.info.json_err, ei.value.info.err_offset) == (e0, off0)


def test_intern_tables_grow():
    """More distinct strings than the first table sizes (set from the record counts) hold: the
    values pass reruns on tables grown 4x until they fit, and the next decode starts from the
    sizes the last one needed; every table equals the oracle's each time."""
    import json as _json
    from kdtn import Engine
    items = []
    for t in range(300):
        links = [{"uid": k, "peer_pod": f"q{t}_{k}", "local_intf": f"e{t}_{k}", "local_ip": f"10.{t % 250}.{k}.1/24",
                  "local_mac": f"02:00:{t // 256:02x}:{t % 256:02x}:{k:02x}:01", "peer_intf": f"f{t}_{k}",
                  "peer_ip": f"10.{t % 250}.{k}.2/24", "peer_mac": f"02:00:{t // 256:02x}:{t % 256:02x}:{k:02x}:02",
                  "properties": {"latency": f"{t * 13 + k}ms", "rate": f"{t * 7 + k}mbit"}} for k in range(12)]
        items.append({"metadata": {"name": f"p{t}", "namespace": "default"}, "spec": {"links": links}})
    doc = _json.dumps({"items": items}).encode()
    eng = Engine(device=0, tick_in_usec=15.625, vxlan_base=5000)
    try:
        for rep in range(2):
            want = check_doc(eng, doc, f"rep {rep}")
            assert want is not None and len(want.kdict.offs) > 24000
        check_doc(eng, b'{"items":[{"metadata":{"name":"a"},"spec":{"links":[{"uid":1,"peer_pod":"b"}]}}]}',
                  "small document after")
    finally:
        eng.close()


def test_depth(engine):
    for d in (15, 16, 17, 40, 9999, 10000, 10001):
        for wrap in (False, True):
            inner = b"[" * d + b"]" * d
            doc = (b'{"items":[{"metadata":{"name":"a","x":' + inner + b'}}]}') if wrap else inner
            check_doc(engine, doc, f"depth {d} wrap {wrap}")
    # deep non-schema structure between links: parents of deep tokens, then schema again
    deep = b'{"k":' + b'{"a":[' * 30 + b'1' + b']}' * 30 + b'}'
    doc = (b'{"items":[{"metadata":{"name":"p","annotations":' + deep + b'},"spec":{"links":[{"uid":1,'
           b'"x":' + deep + b',"peer_pod":"q"},{"uid":2}]}}]}')
    check_doc(engine, doc, "deep")


@pytest.mark.parametrize("lit,want", GO_STRINGS)
def test_go_strings(engine, lit, want):
    doc = b'{"items":[{"metadata":{"name":' + lit + b'}}]}'
    got = check_doc(engine, doc, repr(lit))
    assert got.kdict.get(int(got.topos.name[0])) == want


def test_block_boundaries(engine):
    """quotes, backslash runs, scalars and multi-byte runes straddling 64-byte blocks"""
    rng = random.Random(7)
    for trial in range(40):
        pad = rng.randrange(0, 130)
        s = rng.choice(["a\\\\\\\"b", "\\\\\\\\", "x\\\"y\\\\", "é中😀", "\\u00e9\\ud83d\\ude00", "q" * 70])
        doc = (b'{"items":[{"metadata":{"name":"' + b" " * 0 + b'n' * pad + b'","namespace":"' + s.encode() +
               b'"},"spec":{"links":[{"uid":' + str(rng.randrange(-10**18, 10**18)).encode() +
               b',"properties":{"gap":' + str(rng.randrange(0, 2**32)).encode() + b'}}]}}]}')
        doc = doc.replace(b",", b"," + b" " * rng.randrange(0, 70), rng.randrange(0, 4))
        check_doc(engine, doc, f"trial {trial}")


def test_dense_tokens(engine):
    """waves of more tokens than k_js_tokens lists per wave (TK_MAP = 2048: 64 blocks of "0,")
    around schema values, and one-byte tokens across block and wave edges"""
    for n in (1000, 2100, 5000, 20000):
        arr = b"[" + b",".join([b"0"] * n) + b"]"
        doc = (b'{"items":[{"metadata":{"name":"p","annotations":{"a":' + arr + b'}},"spec":{"links":[{"uid":1,'
               b'"x":' + arr + b',"peer_pod":"q","properties":{"gap":7}},{"uid":2}]}}]}')
        check_doc(engine, doc, f"dense {n}")


def test_many_tiles(engine):
    """a document with > 2 groups of 4096-token tiles (parent scan across groups)"""
    rng = random.Random(11)
    topos = rand_topos(rng, 2500)
    doc = jr.dumps(jr.topology_list(topos, rng, extra=True), rng).encode()
    want = check_doc(engine, doc, "many tiles")
    assert engine._ingest.n_tokens > 2 * 256 * 4096 or want.desired.n > 1000


@pytest.mark.parametrize("tr", range(len(GOLDEN["transitions"])))
def test_samples_chain(engine, tr):
    """config/samples CRs as JSON → GPU ingest → GPU epoch == oracle ingest → oracle epoch"""
    t = GOLDEN["transitions"][tr]
    GOLDEN["sets"].setdefault("S0p", s0p())
    doc = sample_doc(t["status"], t["spec"])
    want = check_doc(engine, doc, t["name"])
    engine.ingest(doc)
    engine.run()
    engine.sync()
    out = engine.download()
    ref = O.reconcile(want, tick=TICK)
    assert not out.mismatches(ref), out.mismatches(ref)


@pytest.mark.parametrize("config", [1, 3, 4])
def test_synthetic_configs(engine, config):
    """synthetic workloads serialised as the API server would, then ingested"""
    kw = dict(pods_per_shard=3000) if config in (3, 4) else {}
    inp = synth.make(config, **kw)
    doc = synth.topology_list_json(inp, pretty=config == 4)
    want = check_doc(engine, doc, f"config {config}")
    # round trip: the strings behind every id equal the generator's
    for k in range(abi.NKEY):
        a = want.desired.key[k][:500]
        assert [want.kdict.get(int(i)) for i in a] == [inp.kdict.get(int(i)) for i in inp.desired.key[k][:500]]
    engine.ingest(doc)
    engine.run()
    engine.sync()
    out = engine.download()
    assert not out.mismatches(O.reconcile(want, tick=TICK))


def test_config2_full_size_whole_document(engine):
    """Config 2 at full size (1M pods, 10M links, 2.86 GB of TopologyList JSON), compared whole:
    every table of the GPU ingest equals the C oracle's decode of the entire document bit for
    bit (first-occurrence dictionaries, topology columns and offsets, the 10M-record store),
    and the epoch the engine runs on its ingested tables equals the oracle's epoch on the
    oracle's own decode (reconcile_parallel: disjoint topology ranges, equal to one call)."""
    inp = synth.make(2, pods_per_shard=1_000_000)
    doc = synth.topology_list_json(inp)
    n_des = inp.desired.n
    del inp
    e0, _, want = O.json_ingest(doc)
    assert e0 == 0 and want.desired.n == n_des == 10_000_000 and want.topos.n == 1_000_000
    info = engine.ingest(doc)
    del doc
    assert (info.n_topos, info.n_desired, info.n_realised) == (1_000_000, n_des, 0)
    tables_equal(engine.ingest_tables(), want, "config 2, whole document")
    engine.run()
    engine.sync()
    out = engine.download()
    bad = out.mismatches(O.reconcile_parallel(want, tick=TICK))
    assert not bad, f"epoch on the ingested tables differs from the oracle in {bad}"


# Scalars and strings far enough from the document end that k_js_validate decides them from
# one 32-byte register window (valid_scalar_window) and one pair of quote/backslash mask
# words (str_end_bs); BAD_SYNTAX's short documents only reach the byte loops.
WIN_SCALARS = [b"0", b"-0", b"7", b"-12", b"0.5", b"-0.25e+3", b"1E9", b"1e-7", b"12345678901234567890",
               b"1.25E+10", b"true", b"false", b"null", b"01", b"-", b"1.", b"1e", b"1e+", b".5", b"+1",
               b"-a", b"1.e3", b"1x", b"0x1", b"truex", b"fals", b"nul", b"nulll", b"tru", b"falsee",
               b"1" * 31, b"1" * 32, b"1" * 40, b"1." + b"5" * 35, b"1e" + b"9" * 33, b"-" + b"0" * 2,
               b"00", b"1.5.2", b"1e5e5", b"1-2", b"NaN", b"Infinity",
               # integer fast paths (digit masks): int64 / uint64 edges, signs, leading zeros
               b"-01", b"-0.0", b"0e0", b"9223372036854775807", b"-9223372036854775808", b"9223372036854775808",
               b"-9223372036854775809", b"18446744073709551615", b"18446744073709551616", b"1" * 19, b"1" * 20,
               b"1" * 21, b"-" + b"1" * 30, b"-" + b"1" * 31, b"4294967295", b"4294967296", b"--1", b"1a"]


@pytest.mark.parametrize("sep", [b"", b" ", b"\t\n"])
def test_window_scalars(engine, sep):
    for s in WIN_SCALARS:
        for pad in (0, 1, 3, 29, 61):
            doc = (b'{"' + b"p" * pad + b'":[' + s + sep + b"]," + b'"q":"' + b"z" * 40 + b'",'
                   b'"items":[{"metadata":{"name":"a"},"spec":{"links":[{"uid":' + s + sep + b"}]}}]}")
            check_doc(engine, doc, f"scalar {s!r} pad {pad}")
            doc = (b'{"' + b"p" * pad + b'":"' + b"z" * 40 + b'",'                      # gap: ParseUint32
                   b'"items":[{"metadata":{"name":"a"},"spec":{"links":[{"uid":1,"properties":{"gap":' + s + sep +
                   b"}}]}}]}")
            check_doc(engine, doc, f"gap {s!r} pad {pad}")


def test_window_strings(engine):
    rng = random.Random(7)
    for L in list(range(0, 70)) + [126, 127, 128, 129, 191, 300]:
        for pad in (0, 1, 62, 63):
            body = bytes(rng.choice(b"abcXYZ019 -") for _ in range(L))
            variants = [body]
            if L >= 2:
                k = rng.randrange(L - 1)
                variants.append(body[:k] + b"\\n" + body[k + 1:])
                variants.append(body[:k] + b"\\q" + body[k + 1:])           # invalid escape
                variants.append(body[:-1] + b"\\\\")                          # escaped backslash at the end
                variants.append(body[:k] + b"\\u00e9" + body[k:])
                variants.append(body[:k] + b'\\"' + body[k:])
            for v in variants:
                doc = (b'{"' + b"p" * pad + b'":"' + v + b'","items":[{"metadata":{"name":"' + v + b'",'
                       b'"namespace":"n"}}], "t":"' + b"w" * 40 + b'"}')
                check_doc(engine, doc, f"string len {L} pad {pad} {v[:20]!r}")


# Member names decoded from their first 17 bytes (key_name's SWAR path) or, with an escape before
# the closing quote, by the byte loop: schema names spelled with escapes, names of 15-18 bytes,
# an escaped quote inside a name, at several alignments.
KEY_VARIANTS = [b"name", b"n\\u0061me", b"na\\u006de", b"\\u006eame", b"namespace", b"namespac\\u0065",
                b"x" * 15, b"x" * 16, b"x" * 17, b"x" * 18, b'na\\"me', b"na\\\\me", b"nam", b"names",
                b"peer_ip", b"peer\\u005fip", b"properties", b"propertie\\u0073", b"properties2", b"uid", b"u\\u0069d"]


def test_window_keys(engine):
    for k in KEY_VARIANTS:
        for pad in (0, 1, 5, 7, 62):
            doc = (b'{"' + b"p" * pad + b'":"z","items":[{"metadata":{"' + k + b'":"a","namespace":"n"},'
                   b'"spec":{"links":[{"' + k + b'":"v","peer_pod":"q","uid":3,"properties":{"' + k +
                   b'":"1ms","latency":"2ms"}}]}}]}')
            check_doc(engine, doc, f"key {k!r} pad {pad}")
