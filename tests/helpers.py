"""Shared test helpers: golden-sample epochs, adversarial random epochs, tricky strings."""
from __future__ import annotations

import random
from fractions import Fraction

import numpy as np

from kdtn import abi
from kdtn.model import Link, LinkProperties, Topology, pack

ACTIONS = {"SKIP": abi.ACT_SKIP, "CREATED": abi.ACT_CREATED, "DIFF": abi.ACT_DIFF}


def links_from(data):
    return [Link.from_dict(d) for d in data]


def golden_epoch(golden, tr):
    """Topologies of one golden transition (status = old set, spec = new set)."""
    sets = golden["sets"]
    topos = []
    for name in ("r1", "r2", "r3"):
        st = None if tr["status"] is None else links_from(sets[tr["status"]][name])
        sp = links_from(sets[tr["spec"]][name])
        pod = golden["pods"][name]
        topos.append(Topology(name, "default", sp, st, pod["src_ip"], pod["net_ns"]))
    return topos


def uids_by_topology(topos, out):
    """{topology: {"action", "del", "add", "upd"}} with uids, from engine/oracle outputs."""
    res = {}
    r0 = n0 = 0
    for t, tp in enumerate(topos):
        st, sp = tp.status_links or [], tp.spec_links or []
        res[tp.name] = {
            "action": int(out.action[t]),
            "del": [st[i - r0].uid for i in out.del_idx[out.del_off[t]:out.del_off[t + 1]]],
            "add": [sp[j - n0].uid for j in out.add_idx[out.add_off[t]:out.add_off[t + 1]]],
            "upd": [sp[j - n0].uid for j in out.upd_idx[out.upd_off[t]:out.upd_off[t + 1]]],
        }
        r0 += len(st)
        n0 += len(sp)
    return res


# ---- adversarial random epochs ---------------------------------------------------------
INTFS = ["eth0", "eth1", "eth2", "veth1", "e"]
IPS = ["", "10.0.0.1/24", "10.0.0.2/24", "10.0.0.3", "300.1.1.1/24", "012.1.1.1/8", "::1/128",
       "fe80::1/64", "1.2.3.4/33", "1.2.3.4/024", "a.b.c.d/1"]
MACS = ["", "00:00:5e:00:53:01", "00-00-5e-00-53-01", "0000.5e00.5301", "00:00-5e:00:53:01",
        "zz:00:5e:00:53:01", "00:00:5e:00:53", "00:00:5e:00:53:01:02:03"]
DURS = ["", "10ms", "1.5s", "0.25ms", "1us", "5m", "1h30m", "10", "-5ms", "1e3ms", "0", "-0",
        ".5s", "1.5µs", "2μs", "3ns", "1h", "9999999999999999999h", "0.000000001ms", "7.0000001s"]
PCTS = ["", "0", "0.1", "25", "99.99999", "100", "100.0", "100.0000001", "101", "-1", "-0",
        "nan", "inf", "1_0", "0x1p-2", "1e1", "abc", "12.5", "33.3", "1e-50", "-1e-50", "+5",
        ".5", "5.", "00.5", "99.999999999999999999999"]
RATES = ["", "1Gbit", "20Mbit", "1000", "1Kibps", "1.5Gbit", " 1gbit ", "bit", "1Kbit", "10TBIT",
         "100mbps", "7Mibit", "0", "18446744073709551615", "18446744073709551616", "1İbit",
         "5Kbit", "12 "]


def random_props(rng: random.Random, p_field=0.35):
    d = {}
    for f in abi.PROP_COLS:
        if rng.random() < p_field:
            if f in ("latency", "jitter"):
                d[f] = rng.choice(DURS)
            elif f == "rate":
                d[f] = rng.choice(RATES)
            else:
                d[f] = rng.choice(PCTS[:12] if rng.random() < 0.7 else PCTS)
    gap = rng.choice([0, 0, 0, 1, 3, 10])
    return LinkProperties.from_dict(dict(d, gap=gap))


def random_epoch(seed: int, T: int = 120, big: int = 0, p_err: float = 0.15):
    """Topologies exercising: nil vs empty lists, duplicates keys/uids, reorders, prop edits,
    invalid CIDR/MAC/props, localhost/physical/missing peers, dead peers, big segments."""
    rng = random.Random(seed)
    names = [f"t{i}" for i in range(T)]
    nss = ["default", "default", "other", ""]
    topos = []
    for i in range(T):
        ns = rng.choice(nss)
        src = rng.choice(["", "10.0.0.1", "10.0.0.2", "10.0.0.3"])
        netns = "" if not src and rng.random() < 0.7 else rng.choice(["/run/ns/a", f"/run/ns/{i}"])
        size = rng.choice([0, 1, 2, 3, 5, 8, 12]) if i >= big else rng.randint(2500, 5200)

        def mk(uid):
            bad = rng.random() < p_err
            return Link(local_intf=rng.choice(INTFS),
                        local_ip=rng.choice(IPS) if bad else rng.choice(IPS[:3]),
                        local_mac=rng.choice(MACS) if bad else rng.choice(MACS[:3]),
                        peer_intf=rng.choice(INTFS),
                        peer_ip=rng.choice(IPS) if bad else rng.choice(IPS[:3]),
                        peer_mac=rng.choice(MACS) if bad else rng.choice(MACS[:2]),
                        peer_pod=rng.choice(names + ["localhost", "physical/1.2.3.4", "ghost", "t0"]),
                        uid=uid, properties=random_props(rng, 0.35 if bad else 0.2))

        old = [mk(rng.randint(1, 40) if size < 100 else rng.randint(1, 10**6)) for _ in range(size)]
        mode = rng.random()
        if mode < 0.15:
            new = [Link(**{**l.__dict__}) for l in old]          # identical → SKIP
        else:
            new = []
            for l in old:
                r = rng.random()
                if r < 0.15:
                    continue                                      # delete
                nl = Link(**{**l.__dict__})
                if r < 0.35:
                    nl.properties = random_props(rng)              # props change
                new.append(nl)
                if rng.random() < 0.05:
                    new.append(Link(**{**nl.__dict__}))           # duplicate key in new
            for _ in range(rng.choice([0, 0, 1, 2])):
                new.append(mk(rng.randint(1, 60)))                # additions
            if rng.random() < 0.3:
                rng.shuffle(new)                                  # reorder (positional ≠)
        if rng.random() < 0.05 and old:
            old.append(Link(**{**old[0].__dict__}))               # duplicate key in old
        st = None if rng.random() < 0.1 else old
        sp = None if rng.random() < 0.08 else new
        topos.append(Topology(names[i], ns, sp, st, src, netns))
    vnis = []
    for _ in range(rng.randint(0, 40)):
        vnis.append((rng.choice(["10.0.0.1", "10.0.0.2", "10.0.0.3"]), 5000 + rng.randint(1, 60),
                     rng.choice(["/run/ns/a", f"/run/ns/{rng.randint(0, T)}", ""])))
    return topos, vnis


def random_epoch_input(seed: int, **kw):
    topos, vnis = random_epoch(seed, **kw)
    return topos, pack(topos, vnis)


# ---- tricky float strings ----------------------------------------------------------------
def exact_decimal(fr: Fraction, max_digits: int = 400) -> str:
    """Exact decimal expansion of a dyadic rational (terminates)."""
    sign = "-" if fr < 0 else ""
    fr = abs(fr)
    ip = fr.numerator // fr.denominator
    rem = fr - ip
    digits = []
    while rem and len(digits) < max_digits:
        rem *= 10
        d = rem.numerator // rem.denominator
        digits.append(str(d))
        rem -= d
    return sign + str(ip) + ("." + "".join(digits) if digits else "")


def midpoint_strings(rng: random.Random, n: int):
    """Decimal strings at/around exact float32 rounding midpoints in [0, 100]."""
    out = []
    for _ in range(n):
        lo = rng.choice([1e-44, 1e-38, 1e-20, 1e-5, 0.001, 0.5, 1.0, 7.0, 33.3, 99.0, 99.9999])
        x = np.float32(rng.uniform(lo, min(100.0, lo * 10 + 1)))
        nx = np.nextafter(x, np.float32(np.inf))
        mid = (Fraction(float(x)) + Fraction(float(nx))) / 2
        s = exact_decimal(mid)
        out.append(s)
        if "." in s:
            out.append(s + "0000001")                    # just above the midpoint
            digs = s.rstrip("0")
            last = digs[-1]
            if last not in ".0":
                out.append(digs[:-1] + str(int(last) - 1) + "9" * rng.randint(1, 30))  # just below
        out.append(s + "e0")
        out.append("0" * rng.randint(0, 5) + s)
    return out


def random_float_strings(rng: random.Random, n: int):
    out = []
    for _ in range(n):
        k = rng.random()
        if k < 0.3:
            ip = str(rng.randint(0, 100))
            fr = "".join(rng.choice("0123456789") for _ in range(rng.randint(0, 30)))
            out.append(ip + ("." + fr if fr or rng.random() < 0.3 else ""))
        elif k < 0.5:
            m = "".join(rng.choice("0123456789") for _ in range(rng.randint(1, 25)))
            e = rng.randint(-60, 5)
            out.append(f"{m[:1]}.{m[1:]}e{e}" if rng.random() < 0.5 else f"{m}E{e:+d}")
        elif k < 0.6:
            out.append(("-" if rng.random() < 0.5 else "") + f"{rng.random() * 1e-40:.30e}")
        elif k < 0.7:
            out.append(f"0x{rng.randint(1, 2**60):x}p{rng.randint(-200, 10)}")
        elif k < 0.8:
            out.append(f"0x{rng.randint(0, 255):x}.{rng.randint(0, 2**40):x}p{rng.randint(-10, 3)}")
        elif k < 0.9:
            s = str(rng.randint(0, 99)) + "." + str(rng.randint(0, 10**8))
            i = rng.randint(0, len(s))
            out.append(s[:i] + "_" + s[i:])
        else:
            out.append("".join(rng.choice("0123456789.eE+-_xXpPinfa") for _ in range(rng.randint(1, 8))))
    return out


# ---- wire-encoding epochs: strings that stress proto.Marshal ---------------------------
def wire_epoch_input(seed: int, T: int = 80):
    """random_epoch plus strings and values that exercise the protobuf encoder: multi-byte
    UTF-8, invalid UTF-8 (Marshal error), strings of 128+ bytes (2-byte length varints),
    negative and large uids (10-byte varints), gaps >= 128."""
    rng = random.Random(seed ^ 0x5A5A)
    topos, vnis = random_epoch(seed, T=T, p_err=0.1)
    uni = ["eth-µ", "veth–1", "日本", "x" * 130, "y" * 300, "🙂pod"]
    bad = [b"\xff", b"ab\xc3", b"\xed\xa0\x80", b"\xc0\xaf", b"\xf4\x90\x80\x80"]
    for t, tp in enumerate(topos):
        if rng.random() < 0.05:
            tp.name = tp.name + rng.choice(uni[:3])
        for side in (tp.spec_links or [], tp.status_links or []):
            for l in side:
                r = rng.random()
                if r < 0.05:
                    l.peer_intf = rng.choice(uni)
                elif r < 0.07:
                    l.local_mac = rng.choice(bad)
                elif r < 0.09:
                    l.properties.rate = rng.choice(uni + [b"1\xffGbit"])
                if rng.random() < 0.05:
                    l.uid = rng.choice([-1, -5, -(2 ** 40), 2 ** 40, 2 ** 62, 127, 128, 16383, 16384])
                if rng.random() < 0.05:
                    l.properties.gap = rng.choice([127, 128, 300, 2 ** 31, 2 ** 32 - 1])
    return topos, pack(topos, vnis)
