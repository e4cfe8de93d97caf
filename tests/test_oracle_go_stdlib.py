"""The oracle's restatements of the Go standard-library parsers on the reconcile path, checked
against the known-answer tables Go publishes with those packages.

The reference calls time.ParseDuration (common/qdisc.go:146-157, via ParseDuration),
net.ParseCIDR and net.ParseMAC (common/veth.go:21-36, MakeVeth) from the Go standard library
(go.mod: go 1.19). Go is absent here and on the GPU box, so the oracle (oracle/kdtn_oracle.c)
restates them; these vectors are the expected values of Go's own package tests — time's
parseDurationTests (time_test.go), net's parseCIDRTests (ip_test.go) and parseMACTests
(mac_test.go) — written out here as data, passed through the reference's wrappers: ParseDuration
rejects a negative duration and returns uint32(d.Microseconds()) (Microseconds truncates toward
zero, uint32 keeps the low 32 bits); "" is 0 without a parse. They pin the restatements to Go's
published answers, not to a run of the reference (parity stays "unpinned" in that sense,
DESIGN.md §6); the GPU parsers are compared with the oracle in tests/test_parity_gpu.py.
"""
import os
import sys

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
