"""Independent decoder + document generator for the CR-ingest parity tests.

`decode(doc)` is a second restatement of what the informer's json.Unmarshal does to a
`TopologyList` (api/v1/topology_types.go:28-176), written on top of Python's own json
parser, so the C oracle (oracle/kdtn_oracle_json.c) is checked against an implementation
that shares none of its code. Python's json agrees with Go's encoding/json on documents
that are valid UTF-8 and carry no lone \\u surrogates (Go maps those to U+FFFD, Python keeps
them); those cases are covered by literal known-answer vectors in tests/test_ingest_cpu.py.

`topology_list(...)` writes TopologyList documents the way the API server serves CRs
(keys in any order, optional whitespace), with knobs for the decoder's corner cases.
"""
from __future__ import annotations

import json
import random

KEYS = ("local_intf", "local_ip", "local_mac", "peer_intf", "peer_ip", "peer_mac", "peer_pod")
PROPS = ("latency", "latency_corr", "jitter", "loss", "loss_corr", "rate", "duplicate",
         "duplicate_corr", "reorder_prob", "reorder_corr", "corrupt_prob", "corrupt_corr")

SYNTAX, DEPTH, TYPE, DUPKEY = 1, 2, 3, 4


class Reject(Exception):
    def __init__(self, code):
        super().__init__(code)
        self.code = code


class Obj(list):
    """A JSON object as its ordered (key, value) pairs (duplicates kept)."""


def _pairs(pairs):
    return Obj(pairs)


class _Interner:
    def __init__(self):
        self.ids = {b"": 0}
        self.strs = [b""]

    def __call__(self, s: str) -> int:
        b = s.encode("utf-8")
        if b not in self.ids:
            self.ids[b] = len(self.strs)
            self.strs.append(b)
        return self.ids[b]


def _obj(v, names):
    """Members of a schema struct as {field: value}; DUPKEY on a repeated schema field."""
    if v is None:
        return None
    if not isinstance(v, Obj):
        raise Reject(TYPE)
    out = {}
    for k, x in v:
        if k in names:
            if k in out:
                raise Reject(DUPKEY)
            out[k] = x
    return out


def _is_obj(v):
    return isinstance(v, Obj)


def decode(doc: bytes):
    """Returns (json_err, tables) with tables a dict of plain Python lists."""
    try:
        root = json.loads(doc.decode("utf-8"), object_pairs_hook=_pairs,
                          parse_constant=lambda c: (_ for _ in ()).throw(ValueError(c)))
    except (ValueError, RecursionError):
        return SYNTAX, None
    kd, pd = _Interner(), _Interner()
    T = {"ns": [], "name": [], "src_ip": [], "net_ns": [], "flags": [], "real_off": [0], "des_off": [0]}
    side = {0: [], 1: []}    # 0 desired, 1 realised: list of (key[7], prop[12], gap, uid)

    def string(v, dct):
        if v is None:
            return 0
        if not isinstance(v, str):
            raise Reject(TYPE)
        return dct(v)

    def int64(v):
        if v is None:
            return 0
        if isinstance(v, bool) or not isinstance(v, int) or not (-2**63 <= v < 2**63):
            raise Reject(TYPE)
        return v

    def uint32(v):
        if v is None:
            return 0
        if isinstance(v, bool) or not isinstance(v, int) or not (0 <= v < 2**32):
            raise Reject(TYPE)
        return v

    def links(v, s, t):
        if v is None:
            return
        if not isinstance(v, list) or _is_obj(v):
            raise Reject(TYPE)
        T["flags"][t] &= ~(2 if s == 0 else 1)
        for el in v:
            key, prop, gap, uid = [0] * 7, [0] * 12, 0, 0
            side[s].append(None)
            slot = len(side[s]) - 1
            if el is not None:
                if not _is_obj(el):
                    raise Reject(TYPE)
                f = _obj(el, set(KEYS) | {"uid", "properties"})
                for k, x in el:                       # document order of the values
                    if k in KEYS:
                        key[KEYS.index(k)] = string(x, kd)
                    elif k == "uid":
                        uid = int64(x)
                    elif k == "properties":
                        p = _obj(x, set(PROPS) | {"gap"})
                        if p is not None:
                            for pk, px in x:
                                if pk in PROPS:
                                    prop[PROPS.index(pk)] = string(px, pd)
                                elif pk == "gap":
                                    gap = uint32(px)
                del f
            side[s][slot] = (key, prop, gap, uid)

    try:
        if root is not None:
            if not _is_obj(root):
                raise Reject(TYPE)
            r = _obj(root, {"items"})
            items = r.get("items")
            if items is not None:
                if not isinstance(items, list) or _is_obj(items):
                    raise Reject(TYPE)
                for it in items:
                    t = len(T["ns"])
                    for c in ("ns", "name", "src_ip", "net_ns"):
                        T[c].append(0)
                    T["flags"].append(3)
                    if it is not None:
                        if not _is_obj(it):
                            raise Reject(TYPE)
                        _obj(it, {"metadata", "spec", "status"})
                        for k, x in it:
                            if k == "metadata":
                                m = _obj(x, {"name", "namespace"})
                                if m is not None:
                                    for mk, mx in x:
                                        if mk == "name":
                                            T["name"][t] = string(mx, kd)
                                        elif mk == "namespace":
                                            T["ns"][t] = string(mx, kd)
                            elif k == "spec":
                                sp = _obj(x, {"links"})
                                if sp is not None and "links" in sp:
                                    links(sp["links"], 0, t)
                            elif k == "status":
                                st = _obj(x, {"links", "src_ip", "net_ns"})
                                if st is not None:
                                    for sk, sx in x:
                                        if sk == "links":
                                            links(sx, 1, t)
                                        elif sk == "src_ip":
                                            T["src_ip"][t] = string(sx, kd)
                                        elif sk == "net_ns":
                                            T["net_ns"][t] = string(sx, kd)
                    T["real_off"].append(len(side[1]))
                    T["des_off"].append(len(side[0]))
    except Reject as e:
        return e.code, None
    return 0, {"topos": T, "desired": side[0], "realised": side[1], "kdict": kd.strs, "pdict": pd.strs}


# ---- document generator ------------------------------------------------------------------
def _ws(rng, p):
    return rng.choice([" ", "\n", "\t", "\r\n  ", ""]) if rng.random() < p else ""


def dumps(v, rng=None, ws=0.0, esc=0.0):
    """json text of v where v uses lists of (key, value) pairs for objects (duplicates and
    order preserved); optional random whitespace and \\u-escaped ASCII in strings."""
    rng = rng or random.Random(0)

    def s(x):
        if isinstance(x, str):
            out = ['"']
            for ch in x:
                o = ord(ch)
                if ch == '"' or ch == "\\":
                    out.append("\\" + ch)
                elif o < 0x20:
                    out.append("\\u%04x" % o)
                elif esc and rng.random() < esc and o < 0x10000:
                    out.append("\\u%04X" % o if rng.random() < 0.5 else "\\u%04x" % o)
                elif esc and rng.random() < esc and ch == "/":
                    out.append("\\/")
                else:
                    out.append(ch)
            out.append('"')
            return "".join(out)
        if x is None:
            return "null"
        if x is True:
            return "true"
        if x is False:
            return "false"
        if isinstance(x, (int, float)):
            return json.dumps(x)
        if isinstance(x, tuple):          # ("raw", text)
            return x[1]
        if isinstance(x, Obj):
            if not x:
                return "{" + _ws(rng, ws) + "}"
            return "{" + _ws(rng, ws) + ("," + _ws(rng, ws)).join(
                s(k) + _ws(rng, ws) + ":" + _ws(rng, ws) + s(val) for k, val in x) + _ws(rng, ws) + "}"
        if isinstance(x, dict):
            return s(Obj(x.items()))
        if isinstance(x, list):
            return "[" + _ws(rng, ws) + ("," + _ws(rng, ws)).join(s(e) for e in x) + _ws(rng, ws) + "]"
        raise TypeError(type(x))
    return _ws(rng, ws) + s(v) + _ws(rng, ws)


def link_obj(l: dict, rng, shuffle=True, extra=False):
    pairs = [(k, l[k]) for k in l if k != "properties"]
    if "properties" in l:
        props = l["properties"]
        if isinstance(props, dict):
            pp = list(props.items())
            if shuffle:
                rng.shuffle(pp)
            props = Obj(pp)
        pairs.append(("properties", props))
    if extra:
        pairs.append(("x-annotation", [Obj([("deep", [[1, 2.5e3, True], Obj([("a", None)])])]), "s"]))
    if shuffle:
        rng.shuffle(pairs)
    return Obj(pairs)


def topology_list(topos, rng=None, shuffle=True, extra=True, managed=True):
    """topos: list of dicts {name, namespace, spec_links (list|None), status_links (list|None),
    src_ip, net_ns, absent: set of field names to omit} (None entries = null items)."""
    rng = rng or random.Random(1)
    items = []
    for t in topos:
        if t is None:
            items.append(None)
            continue
        meta = [("name", t.get("name")), ("namespace", t.get("namespace")),
                ("uid", "0b5ad7a4-%08x" % rng.getrandbits(32)), ("resourceVersion", "12345")]
        if managed:
            meta.append(("managedFields", [Obj([("apiVersion", "y-young.github.io/v1"), ("fieldsType", "FieldsV1"),
                                                ("fieldsV1", Obj([("f:spec", Obj([("f:links", Obj())]))]))])]))
        meta = [p for p in meta if p[1] is not None or rng.random() < 0.5]
        if shuffle:
            rng.shuffle(meta)
        item = Obj([("apiVersion", "y-young.github.io/v1"), ("kind", "Topology"), ("metadata", Obj(meta))])
        if "spec" not in t.get("absent", ()):
            sl = t.get("spec_links")
            item.append(("spec", Obj([("links", None if sl is None else
                                   [None if l is None else link_obj(l, rng, shuffle, extra and rng.random() < 0.1)
                                    for l in sl])])))
        if "status" not in t.get("absent", ()):
            rl = t.get("status_links")
            st = [("skipped", None), ("src_ip", t.get("src_ip")), ("net_ns", t.get("net_ns")),
                  ("links", None if rl is None else
                   [None if l is None else link_obj(l, rng, shuffle) for l in rl])]
            st = [p for p in st if p[1] is not None or p[0] == "links" or rng.random() < 0.5]
            if shuffle:
                rng.shuffle(st)
            item.append(("status", Obj(st)))
        if shuffle:
            rng.shuffle(item)
        items.append(item)
    root = Obj([("apiVersion", "y-young.github.io/v1"), ("items", items), ("kind", "TopologyList"),
                ("metadata", Obj([("resourceVersion", "777"), ("continue", "")]))])
    return root
