"""The oracle's restatements of the Go standard-library parsers on the reconcile path, checked
against the known-answer tables Go publishes with those packages.

The reference calls time.ParseDuration (common/qdisc.go:146-157, via ParseDuration),
strconv.ParseFloat(s, 32) (:128-143, ParseFloatPercentage), strconv.ParseUint(s, 10, 64)
(:162-199, ParseRate), net.ParseCIDR and net.ParseMAC (common/veth.go:21-36, MakeVeth) from the
Go standard library (go.mod: go 1.19). Go is absent here and on the GPU box, so the oracle (oracle/kdtn_oracle.c)
restates them; these vectors are the expected values of Go's own package tests — time's
parseDurationTests (time_test.go), strconv's atof32tests / atoftests (atof_test.go) and
parseUint64Tests (atoi_test.go), net's parseCIDRTests and parseIPTests (ip_test.go) and parseMACTests
(mac_test.go) — written out here as data, passed through the reference's wrappers: ParseDuration
rejects a negative duration and returns uint32(d.Microseconds()) (Microseconds truncates toward
zero, uint32 keeps the low 32 bits); "" is 0 without a parse. They pin the restatements to Go's
published answers, not to a run of the reference (parity stays "unpinned" in that sense,
DESIGN.md §6); the GPU parsers are compared with the oracle in tests/test_parity_gpu.py.
"""
import os
import random
import sys
from fractions import Fraction

import numpy as np
import pytest

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import oracle as O  # noqa: E402

NS, US, MS, S, M, H = 1, 1_000, 1_000_000, 1_000_000_000, 60_000_000_000, 3_600_000_000_000

# time_test.go parseDurationTests: (input, nanoseconds)
GO_DURATIONS = [
    ("0", 0), ("5s", 5 * S), ("30s", 30 * S), ("1478s", 1478 * S),
    ("-5s", -5 * S), ("+5s", 5 * S), ("-0", 0), ("+0", 0),
    ("5.0s", 5 * S), ("5.6s", 5 * S + 600 * MS), ("5.s", 5 * S), (".5s", 500 * MS),
    ("1.0s", 1 * S), ("1.00s", 1 * S), ("1.004s", 1 * S + 4 * MS), ("1.0040s", 1 * S + 4 * MS),
    ("100.00100s", 100 * S + 1 * MS),
    ("10ns", 10 * NS), ("11us", 11 * US), ("12µs", 12 * US), ("12μs", 12 * US), ("13ms", 13 * MS),
    ("14s", 14 * S), ("15m", 15 * M), ("16h", 16 * H),
    ("3h30m", 3 * H + 30 * M), ("10.5s4m", 4 * M + 10 * S + 500 * MS), ("-2m3.4s", -(2 * M + 3 * S + 400 * MS)),
    ("1h2m3s4ms5us6ns", 1 * H + 2 * M + 3 * S + 4 * MS + 5 * US + 6 * NS),
    ("39h9m14.425s", 39 * H + 9 * M + 14 * S + 425 * MS),
    ("52763797000ns", 52763797000 * NS),
    ("0.3333333333333333333h", 20 * M),
    ("9007199254740993ns", (1 << 53) + 1),
    ("9223372036854775807ns", (1 << 63) - 1), ("9223372036854775.807us", (1 << 63) - 1),
    ("9223372036s854ms775us807ns", (1 << 63) - 1),
    ("-9223372036854775808ns", -(1 << 63)), ("-9223372036854775.808us", -(1 << 63)),
    ("-9223372036s854ms775us808ns", -(1 << 63)),
    ("0.100000000000000000000h", 6 * M),
    ("0.830103483285477580700h", 49 * M + 48 * S + 372539827 * NS),
]
# time_test.go parseDurationErrorTests (plus the overflow cases of the same file)
GO_DURATION_ERRORS = ["3", "-", "s", ".", "-.", ".s", "+.s", "1d", "\x85\x85", "\xffff", "hello \xffff world",
                      "9223372036854775810ns", "9223372036854775808ns", "9223372036854775.808us",
                      "9223372036854ms775us808ns", "-9223372036854775809ns"]


def _ref_duration_us(ns: int):
    """ParseDuration (common/qdisc.go:146-157) on Go's answer: (ok, uint32 microseconds)."""
    if ns < 0:
        return False
    return ns // 1000 & 0xFFFFFFFF


@pytest.mark.parametrize("s,ns", GO_DURATIONS)
def test_parse_duration_go_vectors(s, ns):
    want = _ref_duration_us(ns)
    ok, us = O.parse_duration(s)
    if want is False:
        assert not ok, (s, us)
    else:
        assert ok and us == want, (s, ok, us, want)


@pytest.mark.parametrize("s", GO_DURATION_ERRORS)
def test_parse_duration_go_errors(s):
    assert not O.parse_duration(s.encode("latin-1") if "\xff" in s or "\x85" in s else s)[0], s


def test_parse_duration_empty_is_zero():
    assert O.parse_duration("") == (True, 0)          # qdisc.go:148: "" → 0 without a parse


# ip_test.go parseCIDRTests: (input, valid)
GO_CIDRS = [
    ("135.104.0.0/32", True), ("0.0.0.0/24", True), ("135.104.0.0/24", True), ("135.104.0.1/32", True),
    ("135.104.0.1/24", True), ("::1/128", True), ("abcd:2345::/127", True), ("abcd:2345::/65", True),
    ("abcd:2345::/64", True), ("abcd:2345::/63", True), ("abcd:2345::/33", True), ("abcd:2345::/32", True),
    ("abcd:2344::/31", True), ("abcd:2300::/24", True), ("abcd:2345::/24", True), ("2001:DB8::/48", True),
    ("2001:DB8::1/48", True),
    ("192.168.1.1/255.255.255.0", False), ("192.168.1.1/35", False), ("2001:db8::1/-1", False),
    ("2001:db8::1/-0", False), ("-0.0.0.0/32", False), ("0.-1.0.0/32", False), ("0.0.-2.0/32", False),
    ("0.0.0.-3/32", False), ("0.0.0.0/-0", False), ("", False),
    # Go 1.17 and later: an IPv4 octet with a leading zero is rejected
    ("010.0.0.1/8", False), ("1.2.3.04/24", False),
]


@pytest.mark.parametrize("s,valid", GO_CIDRS)
def test_parse_cidr_go_vectors(s, valid):
    assert O.parse_cidr(s) == valid, s


# ip_test.go parseIPTests: (address, valid). ParseCIDR parses the address part with the same
# parseIPv4 / parseIPv6 (Go 1.19 net/ip.go), so each is checked with a prefix length appended
# that is legal for its family ("/24" for dotted quads, "/64" otherwise).
GO_PARSE_IP = [
    ("127.0.1.2", True), ("127.0.0.1", True), ("::ffff:127.1.2.3", True), ("::ffff:7f01:0203", True),
    ("0:0:0:0:0000:ffff:127.1.2.3", True), ("0:0:0:0:000000:ffff:127.1.2.3", True),
    ("0:0:0:0::ffff:127.1.2.3", True), ("2001:4860:0:2001::68", True),
    ("2001:4860:0000:2001:0000:0000:0000:0068", True),
    ("-0.0.0.0", False), ("0.-1.0.0", False), ("0.0.-2.0", False), ("0.0.0.-3", False), ("127.0.0.256", False),
    ("abc", False), ("123:", False), ("fe80::1%lo0", False), ("fe80::1%911", False), ("", False),
    ("a1:a2:a3:a4::b1:b2:b3:b4", False), ("127.001.002.003", False), ("::ffff:127.001.002.003", False),
    ("123.000.000.000", False), ("1.2..4", False), ("0123.0.0.1", False),
]
GO_PARSE_IP_CIDRS = [(ip + ("/24" if "." in ip and ":" not in ip else "/64"), ok) for ip, ok in GO_PARSE_IP]


@pytest.mark.parametrize("s,valid", GO_PARSE_IP_CIDRS)
def test_parse_ip_go_vectors_as_cidrs(s, valid):
    assert O.parse_cidr(s) == valid, s


# mac_test.go parseMACTests: (input, valid)
GO_MACS = [
    ("00:00:5e:00:53:01", True), ("00-00-5e-00-53-01", True), ("0000.5e00.5301", True),
    ("02:00:5e:10:00:00:00:01", True), ("02-00-5e-10-00-00-00-01", True), ("0200.5e10.0000.0001", True),
    ("00:00:00:00:fe:80:00:00:00:00:00:00:02:00:5e:10:00:00:00:01", True),
    ("00-00-00-00-fe-80-00-00-00-00-00-00-02-00-5e-10-00-00-00-01", True),
    ("0000.0000.fe80.0000.0000.0000.0200.5e10.0000.0001", True),
    ("ab:cd:ef:AB:CD:EF", True), ("ab-cd-ef-AB-CD-EF", True), ("abcd.efAB.CDEF", True),
    ("01.02.03.04.05.06", False), ("01:02:03:04:05:06:", False), ("x1:02:03:04:05:06", False),
    ("01002:03:04:05:06", False), ("01:02003:04:05:06", False), ("01:02:03004:05:06", False),
    ("01:02:03:04005:06", False), ("01:02:03:04:05006", False), ("01-02:03:04:05:06", False),
    ("01:02-03-04-05-06", False), ("0123:4567:89AF", False), ("0123-4567-89AF", False),
]


@pytest.mark.parametrize("s,valid", GO_MACS)
def test_parse_mac_go_vectors(s, valid):
    assert O.parse_mac(s) == valid, s


# strconv/atof_test.go atof32tests: (input, Go's answer printed with 'g' -1, or None for ErrRange)
GO_ATOF32 = [
    ("0x1p-100", "7.888609e-31"), ("0x1p100", "1.2676506e+30"),
    # exactly halfway between 1 and the next float32 (ties to even), just below, just above
    ("1.000000059604644775390625", "1"), ("1.000000059604644775390624", "1"),
    ("1.000000059604644775390626", "1.0000001"),
    ("1.000000059604644775390625" + "0" * 10000 + "1", "1.0000001"),
    # the largest float32, and the border above it
    ("340282346638528859811704183484516925440", "3.4028235e+38"),
    ("-340282346638528859811704183484516925440", "-3.4028235e+38"),
    ("0x.ffffffp128", "3.4028235e+38"), ("-0x.ffffffp128", "-3.4028235e+38"),
    ("3.4028236e38", None), ("-3.4028236e38", None), ("0x1.0p128", None), ("-0x1.0p128", None),
    ("3.402823567e38", "3.4028235e+38"), ("-3.402823567e38", "-3.4028235e+38"),
    ("0x.ffffff7fp128", "3.4028235e+38"), ("-0x.ffffff7fp128", "-3.4028235e+38"),
    ("3.4028235678e38", None), ("-3.4028235678e38", None), ("0x.ffffff8p128", None), ("-0x.ffffff8p128", None),
    # subnormals
    ("1e-38", "1e-38"), ("1e-39", "1e-39"), ("1e-40", "1e-40"), ("1e-41", "1e-41"), ("1e-42", "1e-42"),
    ("1e-43", "1e-43"), ("1e-44", "1e-44"), ("6e-45", "6e-45"), ("5e-45", "6e-45"), ("1e-45", "1e-45"),
    ("2e-45", "1e-45"), ("3e-45", "3e-45"),
    ("0x0.89aBcDp-125", "1.2643093e-38"), ("0x0.8000000p-125", "1.1754944e-38"),
    ("0x0.1234560p-125", "1.671814e-39"), ("0x0.1234567p-125", "1.671814e-39"),
    ("0x0.1234568p-125", "1.671814e-39"), ("0x0.1234569p-125", "1.671815e-39"),
    ("0x0.1234570p-125", "1.671815e-39"), ("0x0.0000010p-125", "1e-45"), ("0x0.0000007p-125", "0"),
]
# atoftests (float64) whose answers are float32 values too, so bitSize 32 gives the same answer
GO_ATOF_EXACT = [
    ("1", 1.0), ("+1", 1.0), ("-1", -1.0), ("-0", -0.0), ("625e-3", 0.625),
    ("0x1p0", 1.0), ("0x1p1", 2.0), ("0x1p-1", 0.5), ("0x1ep-1", 15.0), ("-0x1ep-1", -15.0),
    ("-0x1_ep-1", -15.0), ("0x1fFe2.p0", 131042.0), ("0x1fFe2.P0", 131042.0), ("-0x2p3", -16.0),
    ("0x0.fp4", 15.0), ("0x0.fp0", 0.9375),
    ("0", 0.0), ("0e0", 0.0), ("-0e0", -0.0), ("+0e0", 0.0), ("0e-0", 0.0), ("-0e-0", -0.0), ("+0e-0", 0.0),
    ("0e+0", 0.0), ("-0e+0", -0.0), ("+0e+0", 0.0), ("0e+01234567890123456789", 0.0),
    ("0.00e-01234567890123456789", 0.0), ("-0e+01234567890123456789", -0.0),
    ("-0.00e-01234567890123456789", -0.0), ("0x0p+01234567890123456789", 0.0), ("-0x0p+01234567890123456789", -0.0),
    ("1e-4294967296", 0.0), ("1e-18446744073709551616", 0.0), ("0x1p-4294967296", 0.0),
    ("0x1p-18446744073709551616", 0.0),
    ("0x1p+2", 4.0), ("0x.1p+2", 0.25), ("0x1p-2", 0.25), ("0x.1p-2", 0.015625),
    ("1_23.50_0_0e+1_2", 1.235e14), ("0x_1_2.3_4_5p+1_2", 74565.0),
]
GO_ATOF_RANGE = ["1e+4294967296", "1e+18446744073709551616", "0x1p+4294967296", "0x1p+18446744073709551616"]
GO_ATOF_SYNTAX = [
    "", "1x", "1.1.", "0x1e2", "1p2", "1e", "1e-", ".e-1", "1\x00.2", "0x", "0x.", "0x1", "0x.1", "0x1p",
    "0x.1p", "0x1p+", "0x.1p+", "0x1p-", "0x.1p-",
    "-_123.5e+12", "+_123.5e+12", "_123.5e+12", "1__23.5e+12", "123_.5e+12", "123._5e+12", "123.5_e+12",
    "123.5__0e+12", "123.5e_+12", "123.5e+_12", "123.5e_-12", "123.5e-_12", "123.5e+1__2", "123.5e+12_",
    "-_0x12.345p+12", "+_0x12.345p+12", "_0x12.345p+12", "0x__12.345p+12", "0x1__2.345p+12", "0x12_.345p+12",
    "0x12._345p+12", "0x12.3__45p+12", "0x12.345_p+12", "0x12.345p_+12", "0x12.345p+_12", "0x12.345p_-12",
    "0x12.345p-_12", "0x12.345p+1__2", "0x12.345p+12_",
]
GO_ATOF_SPECIAL = ["nan", "NaN", "NAN", "inf", "-Inf", "+INF", "-Infinity", "+INFINITY", "Infinity"]


def _bits(x) -> int:
    return int(np.float32(x).view(np.uint32))


@pytest.mark.parametrize("s,want", GO_ATOF32, ids=[s[:40] for s, _ in GO_ATOF32])
def test_parse_float32_go_atof32_vectors(s, want):
    ok, v = O.parse_float32(s)
    if want is None:
        assert not ok, (s, v)                       # ErrRange
    else:
        assert ok and _bits(v) == _bits(float(want)), (s, v, want)


@pytest.mark.parametrize("s,want", GO_ATOF_EXACT)
def test_parse_float32_go_atof_vectors(s, want):
    ok, v = O.parse_float32(s)
    assert ok and _bits(v) == _bits(want), (s, v, want)


@pytest.mark.parametrize("s", GO_ATOF_RANGE + GO_ATOF_SYNTAX)
def test_parse_float32_go_errors(s):
    assert not O.parse_float32(s)[0], s


def go_percentage(s: str):
    """ParseFloatPercentage (common/qdisc.go:128-143) on Go's ParseFloat(s, 32) answers above:
    None for an error, else the float32 value."""
    if s == "":
        return 0.0
    if s in GO_ATOF_SYNTAX or s in GO_ATOF_RANGE or s in GO_ATOF_SPECIAL:
        return None                                 # syntax / range error, NaN, or ±Inf out of [0, 100]
    table = dict(GO_ATOF32)
    v = float(table[s]) if s in table else dict(GO_ATOF_EXACT)[s]
    if v is None or v < 0 or v > 100:
        return None
    return v


GO_PCT_INPUTS = [s for s, w in GO_ATOF32 if w is not None] + [s for s, _ in GO_ATOF_EXACT] + \
    GO_ATOF_RANGE + GO_ATOF_SYNTAX + GO_ATOF_SPECIAL


@pytest.mark.parametrize("s", GO_PCT_INPUTS, ids=[s[:40] for s in GO_PCT_INPUTS])
def test_parse_percentage_go_vectors(s):
    want = go_percentage(s)
    ok, v = O.parse_pct(s)
    if want is None:
        assert not ok, (s, v)
    else:
        assert ok and (v == want == 0 or _bits(v) == _bits(want)), (s, v, want)


def _f32_exact(a: Fraction, neg: bool):
    """float32 nearest to -a or a (ties to even, subnormals), None past the largest finite."""
    if a == 0:
        return -0.0 if neg else 0.0
    e = a.numerator.bit_length() - a.denominator.bit_length()
    if Fraction(2) ** e > a:
        e -= 1
    unit = Fraction(2) ** max(e - 23, -149)
    q = a / unit
    n = q.numerator // q.denominator
    r = q - n
    if r > Fraction(1, 2) or (r == Fraction(1, 2) and n & 1):
        n += 1
    v = n * unit
    if v >= Fraction(2) ** 128:
        return None
    return -float(v) if neg else float(v)


def test_hex_float32_rounding_exact():
    """Random hexadecimal mantissas across the subnormal, normal and overflow ranges, against
    exact rational rounding (glibc's strtof rounds some hexadecimal subnormals down)."""
    rng = random.Random(11)
    checked = 0
    for _ in range(4000):
        nd = rng.randint(1, 20)
        digs = "".join(rng.choice("0123456789abcdefABCDEF") for _ in range(nd))
        cut = rng.randint(0, nd)
        mant = digs[:cut] + ("." if rng.random() < 0.6 else "") + digs[cut:]
        if mant.strip(".") == "":
            continue
        e = rng.randint(-240, 140)
        sign = rng.choice(["", "-", "+"])
        s = f"{sign}0x{mant}p{e}"
        ip, _, fp = mant.partition(".")
        fr = Fraction(int(ip or "0", 16) * 16 ** len(fp) + int(fp or "0", 16), 16 ** len(fp)) * Fraction(2) ** e
        want = _f32_exact(fr, sign == "-")
        ok, v = O.parse_float32(s)
        if want is None:
            assert not ok, (s, v)
        else:
            assert ok and _bits(v) == _bits(want), (s, v, want)
        checked += 1
    assert checked > 3500


# strconv/atoi_test.go parseUint64Tests (base 10): (input, value or None for an error), through
# ParseRate (common/qdisc.go:162-199), whose unit stripping leaves these strings unchanged:
# "" is 0 without a parse (:164-166), the rest go to ParseUint(rate, 10, 64) × 1.
GO_PARSE_UINT64 = [
    ("", 0), ("0", 0), ("1", 1), ("12345", 12345), ("012345", 12345), ("12345x", None),
    ("98765432100", 98765432100), ("18446744073709551615", (1 << 64) - 1),
    ("18446744073709551616", None), ("18446744073709551620", None),
    ("1_2_3_4_5", None), ("_12345", None), ("1__2345", None), ("12345_", None),
    ("-0", None), ("-1", None), ("+1", None),
]


@pytest.mark.parametrize("s,want", GO_PARSE_UINT64)
def test_parse_rate_go_parse_uint_vectors(s, want):
    ok, v = O.parse_rate(s)
    if want is None:
        assert not ok, (s, v)
    else:
        assert ok and v == want, (s, v, want)


# strings_test.go trimSpaceTests with the payload made numeric ("abc" -> "123", "x" -> "7",
# "y" -> "8"): ParseRate (common/qdisc.go:163) trims with strings.TrimSpace (unicode.IsSpace:
# "\t\v\r\f\n", U+0085, U+00A0, U+2000, U+3000 ...) after strings.ToLower, then ParseUint's
# answer on what TrimSpace leaves: (input, rate or None for an error).
_GO_SPACE = "\t\v\r\f\n\u0085\u00a0\u2000\u3000"
GO_TRIMSPACE_RATES = [
    ("", 0), ("123", 123), (_GO_SPACE + "123" + _GO_SPACE, 123), (" ", 0), (" \t\r\n \t\t\r\r\n\n ", 0),
    (" \t\r\n 7\t\t\r\r\n\n ", 7), (" \u2000\t\r\n 7\t\t\r\r\n8\n \u3000", None), ("1 \t\r\n2", None),
    (" 7\x80", None), (" 7\xc0", None), ("7 \xc0\xc0 ", None), ("7 \xc0", None), ("7 ☺ ", None),
]


def _latin1_or_utf8(s: str) -> bytes:
    """The test strings' bytes: \x80 / \xc0 stand for single invalid UTF-8 bytes, as in Go."""
    out = bytearray()
    for ch in s:
        out += bytes([ord(ch)]) if ch in "\x80\xc0" else ch.encode()
    return bytes(out)


@pytest.mark.parametrize("s,want", GO_TRIMSPACE_RATES)
def test_parse_rate_go_trimspace_vectors(s, want):
    ok, v = O.parse_rate(_latin1_or_utf8(s))
    if want is None:
        assert not ok, (s, v)
    else:
        assert ok and v == want, (s, v, want)
