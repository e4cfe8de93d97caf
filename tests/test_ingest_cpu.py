"""CR ingest on the CPU: the C oracle's TopologyList decode
(oracle/kdtn_oracle_json.c) against an independent decoder built on Python's json
(tests/json_ref.py), against literal known answers for the Go-specific string rules, and
end to end from the reference's own sample CRs (config/samples, via tests/golden/samples.json)
through the oracle reconcile to the hand-derived transitions.
"""
from __future__ import annotations

import json
import os
import random
import sys

import numpy as np
import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(os.path.dirname(HERE), "oracle"))
sys.path.insert(0, HERE)

import oracle  # noqa: E402
import json_ref as jr  # noqa: E402
from json_ref import Obj  # noqa: E402

GOLDEN = json.load(open(os.path.join(HERE, "golden", "samples.json")))


def as_lists(inp):
    """oracle EpochInput → the json_ref.decode table shape"""
    T = inp.topos
    topos = {"ns": T.ns.tolist(), "name": T.name.tolist(), "src_ip": T.src_ip.tolist(),
             "net_ns": T.net_ns.tolist(), "flags": T.flags.tolist(),
             "real_off": T.real_off.tolist(), "des_off": T.des_off.tolist()}

    def recs(L):
        return [(L.key[:, i].tolist(), L.prop[:, i].tolist(), int(L.gap[i]), int(L.uid[i]))
                for i in range(L.n)]
    return {"topos": topos, "desired": recs(inp.desired), "realised": recs(inp.realised),
            "kdict": [inp.kdict.get(i) for i in range(inp.kdict.n)],
            "pdict": [inp.pdict.get(i) for i in range(inp.pdict.n)]}


def both(doc: bytes):
    e1, _, inp = oracle.json_ingest(doc)
    e2, ref = jr.decode(doc)
    return e1, (as_lists(inp) if inp is not None else None), e2, ref


WORDS = ["eth0", "eth1", "r1", "r2", "default", "kube-system", "10.0.0.1/24", "12.12.12.2/24",
         "00:00:5e:00:53:01", "physical/10.1.1.1", "localhost", "é", "中文", "😀x", "a\"b", "a\\b",
         "tab\there", "/run/netns/r1", "", "10ms", "0.5", "1Gbit", "100Mibps", "1.5s", "99.9",
         # around the GPU's 32-byte string window: equal prefixes, last-byte differences
         "x" * 31, "x" * 32, "x" * 33, "x" * 31 + "y", "x" * 32 + "y", "x" * 64,
         "/run/netns/cni-0123456789abcdef0", "/run/netns/cni-0123456789abcdef1",
         "/run/netns/cni-0123456789abcde", "/run/netns/cni-0123456789abcdf"]


def rand_link(rng):
    l = {}
    for k in jr.KEYS:
        if rng.random() < 0.7:
            l[k] = rng.choice(WORDS)
    if rng.random() < 0.8:
        l["uid"] = rng.choice([0, 1, 7, -3, 2**63 - 1, -2**63, rng.randrange(1 << 40)])
    if rng.random() < 0.7:
        p = {}
        for k in jr.PROPS:
            if rng.random() < 0.3:
                p[k] = rng.choice(WORDS)
        if rng.random() < 0.3:
            p["gap"] = rng.choice([0, 1, 4294967295, None])
        l["properties"] = p if rng.random() < 0.9 else None
    return l


def rand_topos(rng, n):
    out = []
    for t in range(n):
        if rng.random() < 0.05:
            out.append(None)
            continue
        d = {"name": rng.choice(WORDS + ["p%d" % t]), "namespace": rng.choice(["default", "ns1", "", None]),
             "src_ip": rng.choice(["10.0.0.1", "10.0.0.2", "", None]),
             "net_ns": rng.choice(["/run/netns/a", "", None]),
             "absent": set(rng.sample(["spec", "status"], rng.choice([0, 0, 0, 1])))}
        for side in ("spec_links", "status_links"):
            r = rng.random()
            d[side] = None if r < 0.15 else [None if rng.random() < 0.03 else rand_link(rng)
                                              for _ in range(rng.choice([0, 1, 2, 5, 12]))]
        out.append(d)
    return out


@pytest.mark.parametrize("seed", range(12))
def test_oracle_matches_python_json(seed):
    rng = random.Random(seed)
    root = jr.topology_list(rand_topos(rng, 40), rng)
    doc = jr.dumps(root, rng, ws=0.2 if seed % 2 else 0.0, esc=0.05 if seed % 3 == 0 else 0.0).encode()
    e1, a, e2, b = both(doc)
    assert e1 == e2 == 0
    assert a == b


def test_empty_and_null_shapes():
    for doc, T in [(b"null", 0), (b"{}", 0), (b'{"items":null}', 0), (b'{"items":[]}', 0),
                   (b' {"items":[null,{}]} ', 2), (b'{"items":[{"spec":null,"status":null}]}', 1)]:
        e1, a, e2, b = both(doc)
        assert e1 == e2 == 0, doc
        assert a == b and len(a["topos"]["ns"]) == T, doc
        assert all(f == 3 for f in a["topos"]["flags"])
    e, _, inp = oracle.json_ingest(b'{"items":[{"spec":{"links":[]},"status":{"links":[null]}}]}')
    assert e == 0 and inp.topos.flags.tolist() == [0] and inp.realised.n == 1 and inp.desired.n == 0


BAD_SYNTAX = [b"", b" ", b"{", b"}", b"[1,]", b'{"a":1,}', b'{"a" 1}', b'{"a":}', b"{'a':1}", b"01",
              b"-", b"1.", b"1e", b".5", b"+1", b"tru", b"nul", b'"abc', b'"a\\x"', b'"\\u12G4"',
              b'"a\x01b"', b"[1 2]", b'{"items":[]} x', b"[]]", b"[[]", b'{"a":1 "b":2}', b"[,]",
              b'{"items":[{"spec":{"links":[{"uid":1}]}}]', b"\xef\xbb\xbf{}", b"NaN", b"[1,\x0b2]",
              # separators (no tokens of their own on the GPU: recorded on the token after them)
              ] + [b",", b" , ", b":", b",[]", b"[],", b"[]:", b"[1,,2]", b"[1::2]", b"[1 :2]", b"[,1]", b"[:1]",
              b'{"a"::1}', b'{"a":1,,"b":2}', b'{,"a":1}', b'{:"a":1}', b'{"a",1}', b'{"a":1:2}', b"[1,",
              b"[1, ", b'{"a":', b'{"a" : ', b'{"a":1,', b'{"a" :, }', b"[{}:1]", b'{"a":{},:1}', b"[[]:]",
              b'{"a":1}, {"b":2}', b'{"a":1 , , }', b'{"a"', b'["a",', b'{"a":[1,2],}']
SEP_SYNTAX = BAD_SYNTAX[BAD_SYNTAX.index(b","):]


@pytest.mark.parametrize("doc", BAD_SYNTAX)
def test_syntax_errors(doc):
    e1, _, _ = oracle.json_ingest(doc)
    assert e1 == jr.SYNTAX
    try:
        e2, _ = jr.decode(doc)
    except UnicodeDecodeError:
        e2 = jr.SYNTAX
    assert e2 == jr.SYNTAX


# Bad escapes with the offset Go's scanner reports (encoding/json scanner.go: checkValid stops
# at the byte a step rejects; stateInStringEsc rejects the escape byte, stateInStringEscU* the
# first non-hex digit; SyntaxError.Offset counts the bytes read, the rejected one included, so
# the 0-based index here is Offset - 1; an escape cut by the document's end is "unexpected end
# of JSON input" at len(data)). Derived by hand from those state functions, byte by byte.
GO_ESCAPE_OFFSETS = [
    (b'"a\\x"', 3),                       # 'x' after the backslash
    (b'["\\u12G4"]', 6),                  # 'G', the third hex digit
    (b'{"a\\q":1}', 4),                   # 'q'
    (b'["ok", "b\\\\\\z"]', 12),        # a run of three: the third backslash escapes 'z'
    (b'["\\u12"]', 6),                    # the closing quote is no hex digit
    (b'{"items":[{"metadata":{"name":"' + b"x" * 70 + b'\\u00zz"}}]}', 105),   # crosses a 64-B block
    (b'["\\u1', 5),                       # cut by the end
    (b'"ab\\', 4),
    (b'"' + b"\\\\" * 40 + b'\\e"', 82),  # an even run of 80 over two blocks, then a bad escape
]


@pytest.mark.parametrize("doc,off", GO_ESCAPE_OFFSETS)
def test_escape_error_offsets_go_semantics(doc, off):
    e, o, _ = oracle.json_ingest(doc)
    assert (e, o) == (oracle.JSON_SYNTAX if hasattr(oracle, "JSON_SYNTAX") else 1, off)


def test_depth_limit():
    ok = b"[" * 10000 + b"]" * 10000
    deep = b"[" * 10001 + b"]" * 10001
    assert oracle.json_ingest(ok)[0] == 0 or oracle.json_ingest(ok)[0] == jr.TYPE
    assert oracle.json_ingest(deep)[0] == jr.DEPTH
    # depth is counted through unknown fields too
    d = b'{"x":' + b"[" * 9999 + b"]" * 9999 + b"}"
    assert oracle.json_ingest(d)[0] == 0
    d = b'{"x":' + b"[" * 10000 + b"]" * 10000 + b"}"
    assert oracle.json_ingest(d)[0] == jr.DEPTH


TYPE_ERRORS = [
    b"[]", b'"x"', b"5", b'{"items":{}}', b'{"items":5}', b'{"items":[5]}', b'{"items":["a"]}',
    b'{"items":[{"metadata":[]}]}', b'{"items":[{"metadata":{"name":5}}]}',
    b'{"items":[{"metadata":{"namespace":true}}]}', b'{"items":[{"spec":[]}]}',
    b'{"items":[{"spec":{"links":{}}}]}', b'{"items":[{"spec":{"links":[1]}}]}',
    b'{"items":[{"status":{"src_ip":1}}]}', b'{"items":[{"status":{"links":"x"}}]}',
    b'{"items":[{"spec":{"links":[{"uid":1.5}]}}]}', b'{"items":[{"spec":{"links":[{"uid":1e2}]}}]}',
    b'{"items":[{"spec":{"links":[{"uid":"1"}]}}]}', b'{"items":[{"spec":{"links":[{"uid":9223372036854775808}]}}]}',
    b'{"items":[{"spec":{"links":[{"uid":-9223372036854775809}]}}]}',
    b'{"items":[{"spec":{"links":[{"local_ip":["a"]}]}}]}',
    b'{"items":[{"spec":{"links":[{"properties":[]}]}}]}',
    b'{"items":[{"spec":{"links":[{"properties":{"gap":-1}}]}}]}',
    b'{"items":[{"spec":{"links":[{"properties":{"gap":4294967296}}]}}]}',
    b'{"items":[{"spec":{"links":[{"properties":{"gap":1.0}}]}}]}',
    b'{"items":[{"spec":{"links":[{"properties":{"rate":100}}]}}]}',
    b'{"items":[{"spec":{"links":[{"uid":12345678901234567890123456789012345}]}}]}',
    b'{"items":[{"spec":{"links":[{"uid":-1234567890123456789012345678901234}]}}]}',
    b'{"items":[{"spec":{"links":[{"properties":{"gap":123456789012345678901234567890123}}]}}]}',
    b'{"items":[{"spec":{"links":[{"uid":18446744073709551616}]}}]}',
    b'{"items":[{"spec":{"links":[{"properties":{"gap":18446744073709551615}}]}}]}',
]


@pytest.mark.parametrize("doc", TYPE_ERRORS)
def test_type_errors(doc):
    assert oracle.json_ingest(doc)[0] == jr.TYPE
    assert jr.decode(doc)[0] == jr.TYPE


DUPS = [b'{"items":[],"items":[]}', b'{"items":[{"spec":{},"spec":{}}]}',
        b'{"items":[{"metadata":{"name":"a","name":"b"}}]}',
        b'{"items":[{"spec":{"links":[{"uid":1,"uid":2}]}}]}',
        b'{"items":[{"spec":{"links":[{"properties":{"gap":1,"gap":1}}]}}]}',
        b'{"items":[{"status":{"net_ns":"a","net_ns":null}}]}']


@pytest.mark.parametrize("doc", DUPS)
def test_duplicate_schema_fields(doc):
    assert oracle.json_ingest(doc)[0] == jr.DUPKEY
    assert jr.decode(doc)[0] == jr.DUPKEY


def test_unknown_fields_are_skipped():
    doc = (b'{"kind":"TopologyList","items":[{"kind":1,"apiVersion":[{}],"metadata":{"name":"a",'
           b'"labels":{"x":"y"},"NAME":"b","Name":"c"},"spec":{"Links":[1],"links":[]},'
           b'"status":{"skipped":["x"],"links":null,"extra":{"links":7}}}],"metadata":{}}')
    e, _, inp = oracle.json_ingest(doc)
    assert e == 0
    assert inp.kdict.get(int(inp.topos.name[0])) == b"a"       # case-sensitive keys
    assert inp.topos.flags.tolist() == [1]                       # spec links [], status nil
    # keys whose escapes decode to a schema name match it
    e, _, inp = oracle.json_ingest(b'{"items":[{"metadata":{"n\\u0061me":"z"}}]}')
    assert e == 0 and inp.kdict.get(int(inp.topos.name[0])) == b"z"


# Go-specific string decoding (encoding/json unquote): literal known answers
GO_STRINGS = [
    (b'"\\ud83d\\ude00"', "😀".encode()),                     # surrogate pair
    (b'"\\ud83dx"', b"\xef\xbf\xbdx"),                          # lone high surrogate → U+FFFD
    (b'"\\ude00"', b"\xef\xbf\xbd"),                            # lone low surrogate
    (b'"\\ud83d\\u0041"', b"\xef\xbf\xbdA"),                    # high + non-low: both decoded alone
    (b'"\\ud83d\\ud83d\\ude00"', b"\xef\xbf\xbd" + "😀".encode()),
    (b'"a\xffb"', b"a\xef\xbf\xbdb"),                           # invalid UTF-8 byte → U+FFFD
    (b'"\xc3\xa9"', "é".encode()),                              # valid UTF-8 kept
    (b'"\xc3"', b"\xef\xbf\xbd"),                               # truncated sequence
    (b'"\xed\xa0\x80"', b"\xef\xbf\xbd" * 3),                   # UTF-8-encoded surrogate
    (b'"\xe0\x80\x80"', b"\xef\xbf\xbd" * 3),                   # overlong
    (b'"\\u00e9\\/\\b\\f\\n\\r\\t\\"\\\\"', "é/\b\f\n\r\t\"\\".encode()),
    (b'"\\u0000"', b"\x00"),
]


@pytest.mark.parametrize("lit,want", GO_STRINGS)
def test_go_string_decoding(lit, want):
    doc = b'{"items":[{"metadata":{"name":' + lit + b'}}]}'
    e, _, inp = oracle.json_ingest(doc)
    assert e == 0
    assert inp.kdict.get(int(inp.topos.name[0])) == want


def sample_doc(status_set, spec_set, rng=None, **kw):
    """TopologyList of the reference's sample topologies r1..r3 (config/samples) with
    status.links from one link set and spec.links from another (None = nil)."""
    sets = GOLDEN["sets"]
    topos = []
    for name in ("r1", "r2", "r3"):
        topos.append({"name": name, "namespace": "default",
                      "src_ip": GOLDEN["pods"][name]["src_ip"], "net_ns": GOLDEN["pods"][name]["net_ns"],
                      "spec_links": sets[spec_set][name],
                      "status_links": None if status_set is None else sets[status_set][name]})
    return jr.dumps(jr.topology_list(topos, rng or random.Random(3), **kw), rng or random.Random(4), ws=0.1).encode()


def s0p():
    s0 = json.loads(json.dumps(GOLDEN["sets"]["S0"]))
    s0["r1"] = [l for l in s0["r1"] if l["uid"] != 2] + [
        {"uid": 4, "peer_pod": "r3", "local_intf": "eth3", "peer_intf": "eth3",
         "local_ip": "14.14.14.1/24", "peer_ip": "14.14.14.3/24"}]
    return s0


@pytest.mark.parametrize("tr", range(len(GOLDEN["transitions"])))
def test_samples_ingest_then_reconcile(tr):
    """config/samples CRs as JSON → ingest → oracle reconcile → the hand-derived
    transitions of SURVEY Appendix B (tests/golden/samples.json)."""
    t = GOLDEN["transitions"][tr]
    GOLDEN["sets"].setdefault("S0p", s0p())
    doc = sample_doc(t["status"], t["spec"])
    e1, a, e2, b = both(doc)
    assert e1 == e2 == 0 and a == b
    _, _, inp = oracle.json_ingest(doc)
    out = oracle.reconcile(inp)
    names = [inp.kdict.get(int(i)).decode() for i in inp.topos.name]
    act = {0: "SKIP", 1: "CREATED", 2: "DIFF"}
    for ti, name in enumerate(names):
        exp = t["expect"][name]
        assert act[int(out.action[ti])] == exp["action"]
        for lst, L, off in (("del", inp.realised, out.del_off), ("add", inp.desired, out.add_off),
                            ("upd", inp.desired, out.upd_off)):
            idx = getattr(out, lst + "_idx")[off[ti]:off[ti + 1]]
            assert [int(L.uid[i]) for i in idx] == exp[lst], (name, lst)


def test_window_scalars_oracle_pinned():
    """the oracle's checkValid on the GPU window cases agrees with Python's json"""
    import test_ingest_gpu as g
    for s in g.WIN_SCALARS:
        doc = b'{"p":[' + s + b'],"q":"' + b"z" * 40 + b'"}'
        e1, _, _ = oracle.json_ingest(doc)
        try:
            json.loads(doc, parse_constant=lambda c: (_ for _ in ()).throw(ValueError(c)))
            std_ok = True
        except ValueError:
            std_ok = False
        assert (e1 != jr.SYNTAX) == std_ok, (s, e1)


def test_schema_name_hash_is_perfect():
    """k_js_values looks member names up by a 7-bit hash of their zero-padded 16 bytes
    (kdtn_ingest.hip: kAll / name_hash): the 31 schema names must land in distinct slots"""
    import re
    import struct
    from pathlib import Path
    src = (Path(__file__).resolve().parents[1] / "kube-dtn_amd" / "csrc" / "kdtn_ingest.hip").read_text()
    table = src[src.index("kAll[KN_ALL][16] = {"):]
    names = re.findall(r'"([a-z_]+)"', table[:table.index("};")])
    k1, k2 = (int(x, 16) for x in re.findall(r"\* (0x[0-9A-F]+)ull", src[src.index("uint32_t name_hash"):])[:2])
    m = (1 << 64) - 1
    slots = set()
    for n in names:
        lo, hi = struct.unpack("<QQ", n.encode().ljust(16, b"\0"))
        slots.add((((lo ^ ((hi * k1) & m)) * k2) & m) >> 57)
    assert len(names) == 31 and len(slots) == 31
