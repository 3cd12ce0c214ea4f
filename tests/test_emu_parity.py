"""CPU parity of the device per-line logic (lp_device.h compiled for the host
by the test-only tests/emu build) against the oracle.  The same comparisons
run on the real GPU path in test_gpu_parity.py."""
import json
import random

import pytest

import golden_check
import logparser_amd as lpa

ALL = None


def all_paths(oracle):
    global ALL
    if ALL is None:
        ALL = oracle.possible_paths("combined")
    return ALL


def compare(o, e, lines, allow_fallback=True):
    stats = {"ok": 0, "bad": 0, "fallback": 0}
    for l in lines:
        s1, r1 = o.parse_raw(l)
        s2, r2 = e.parse_raw(l)
        assert s2 != 3, r2  # arena overflow would be a sizing bug
        if s2 == 2:
            stats["fallback"] += 1
            assert allow_fallback, l
            continue
        if s1 == 2:
            pytest.fail("device decided a line the oracle cannot restate: %r" % l)
        assert s1 == s2, (l, s1, s2)
        if s1 == 0:
            assert r1 == r2, (l, json.dumps(json.loads(r1), indent=0)[:2000], r2[:2000])
            stats["ok"] += 1
        else:
            stats["bad"] += 1
    return stats


def test_golden_vectors_emulated(oracle, emu, vectors):
    n_checked = 0
    for c in vectors["cases"]:
        e = emu.Emu(c["logformat"], c["fields"], c["remaps"])
        if e.status != 0:  # not on the device: every line FALLBACK
            assert e.parse(c["line"])[0] == 2
            continue
        st, rec = e.parse(c["line"])
        if st == 2:
            continue
        assert golden_check.check_case(c, st, rec or {}) == [], c["source"]
        n_checked += 1
    assert n_checked >= 30


def test_demolog_emulated(oracle, emu, demolog_lines):
    o = oracle.Oracle("combined", all_paths(oracle))
    e = emu.Emu("combined", all_paths(oracle))
    s = compare(o, e, demolog_lines)
    assert s["ok"] + s["fallback"] == 3456 and s["fallback"] < 30, s


def test_synthetic_config2_emulated(oracle, emu):
    data = lpa.synth_combined(20261015, 0, 5000)
    lines = data.split(b"\n")[:-1]
    o = oracle.Oracle("combined", all_paths(oracle))
    e = emu.Emu("combined", all_paths(oracle))
    s = compare(o, e, lines, allow_fallback=False)
    assert s["ok"] == 5000


def mutate(rng, line):
    ops = [
        lambda l: l[: rng.randrange(len(l))],                      # truncated
        lambda l: l.replace(b'"', b"", 1),                          # missing quote
        lambda l: l.replace(b"/Jan/", b"/Foo/").replace(b"/Feb/", b"/Foo/").replace(b"/Mar/", b"/Foo/"),
        lambda l: l.replace(b"[0", b"[00", 1)[:-1] if b"[0" in l else l,
        lambda l: l.replace(b" 200 ", b" 200 x", 1),
        lambda l: l + b" extra",
        lambda l: l.replace(b"GET /", b"GET /a b/", 1),             # space in URI
        lambda l: l.replace(b"?", b"?x=%zz&", 1),                   # bad escape
        lambda l: l.replace(b"/", b"/#frag", 1),
        lambda l: l.replace(b"HTTP/1.1", b"HTTP/1", 1),
        lambda l: l.replace(b"http://", b"http://user@", 1),
        lambda l: l.replace(b"https://", b"ht tps://", 1),
        lambda l: l.replace(b"=", b"=%u0041", 1),
        lambda l: l.replace(b" - - ", b" 12 - ", 1),
        lambda l: l.replace(b"+0", b"-1", 1),
        lambda l: l.replace(b"&", b"&amp;", 1),
        lambda l: l.replace(b"1", b"\t", 1),
        lambda l: l.replace(b"a", b"\xc3\xa9", 1),
        # URI / query corner cases
        lambda l: l.replace(b"?", b"?Upper=X&", 1),
        lambda l: l.replace(b"?", b"?a b=c d&", 1),
        lambda l: l.replace(b"=", b"=x+y%41%e9", 1),
        lambda l: l.replace(b"&", b"?", 1),
        lambda l: l.replace(b"?", b"?x=1&amp;y=2&", 1),
        lambda l: l.replace(b"?", b"?q=a;b&", 1),
        lambda l: l.replace(b"?", b"?&&=&", 1),
        lambda l: l.replace(b" HTTP/", b"#frag%41?x&y HTTP/", 1),
        lambda l: l.replace(b" HTTP/", b"#a HTTP/", 1),
        lambda l: l.replace(b"GET /", b"GET /%7Epath%2Fx/", 1),
        lambda l: l.replace(b"GET /", b"GET /a{b}|c^/", 1),
        lambda l: l.replace(b"GET /", b"GET /p\"q/", 1),
        lambda l: l.replace(b"?", b"?N%41ME=1&", 1),
        lambda l: l.replace(b"http://", b"http://Host-Name.EXAMPLE:8080", 1),
        lambda l: l.replace(b"://", b"://1.2.3.4:0", 1),
        lambda l: l.replace(b"://", b"://[::1]", 1),
        lambda l: l.replace(b"?", b"?=v&k&", 1),
        lambda l: l.replace(b"GET /", b"GET //double/", 1),
    ]
    return rng.choice(ops)(line)


def test_mutated_lines_emulated(oracle, emu):
    rng = random.Random(1234)
    base = lpa.synth_combined(99, 0, 3000).split(b"\n")[:-1]
    lines = [mutate(rng, l) for l in base] + [mutate(rng, mutate(rng, l)) for l in base]
    o = oracle.Oracle("combined", all_paths(oracle))
    e = emu.Emu("combined", all_paths(oracle))
    s = compare(o, e, lines)
    assert s["bad"] > 50 and s["ok"] > 50, s


@pytest.mark.parametrize("fmt", ["common", "combinedio", "%h %l %u %t \"%r\" %>s %b", "%a %A %{Host}i %u %t %r"])
def test_other_formats_emulated(oracle, emu, fmt):
    paths = oracle.possible_paths(fmt)
    o = oracle.Oracle(fmt, paths)
    e = emu.Emu(fmt, paths)
    if e.status != 0:
        pytest.skip("not on device: " + e.err)
    rng = random.Random(5)
    lines = []
    for l in lpa.synth_combined(3, 0, 300).split(b"\n")[:-1]:
        lines.append(l)
        lines.append(mutate(rng, l))
    compare(o, e, lines)


def test_lines_in_batch_context_emulated(oracle, emu, vectors, demolog_lines):
    """Lines parsed in place inside a whole batch buffer (arbitrary 4-byte
    phase, neighbouring lines' bytes in the scanned words) give the same
    records as lines parsed alone."""
    groups = {}
    for c in vectors["cases"]:
        groups.setdefault((c["logformat"], tuple(c["fields"]), tuple(map(tuple, c["remaps"]))), []).append(
            c["line"].encode())
    groups[("combined", tuple(all_paths(oracle)), ())] = demolog_lines[:400] + lpa.synth_combined(8, 0, 400).split(b"\n")[:-1]
    for (fmt, fields, remaps), lines in groups.items():
        e = emu.Emu(fmt, list(fields), list(remaps))
        if e.status != 0:
            continue
        for pad in range(4):
            data = b"x" * pad + b"\n" + b"\n".join(lines) + b"\n"
            got = e.parse_batch_raw(data)[1:]
            assert len(got) == len(lines)
            for l, (st, js) in zip(lines, got):
                assert (st, js) == e.parse_raw(l), (fmt, l)


NGINX = lpa.SYNTH_FORMATS[lpa.SYNTH_NGINX]


def mutate_nginx(rng, line):
    """Config-4 corner cases: upstream lists (UpstreamModule.upstreamListOf),
    SECOND_MILLIS values, the strict 3-part $request, $pipe."""
    ops = [
        lambda l: l.replace(b" .", b" p", 1),
        lambda l: l[:-1] + b"..",                                     # $pipe is one char
        lambda l: l.replace(b" HTTP/", b" x HTTP/", 1),               # 4-part request: no match
        lambda l: l.replace(b'"GET ', b'"GET  ', 1),
        lambda l: l.rsplit(b" ", 2)[0] + b" 0.002, 0.003 : 0.004 .",
        lambda l: l.rsplit(b" ", 2)[0] + b" 0.002 , 0.003 .",
        lambda l: l.rsplit(b" ", 2)[0] + b" 0.002,0.003 .",           # not split by ', ': FALLBACK
        lambda l: l.rsplit(b" ", 2)[0] + b" 0.002 : 0.003 .",
        lambda l: l.rsplit(b" ", 2)[0] + b" - .",                     # '-' is not a SECOND_MILLIS
        lambda l: l.rsplit(b" ", 2)[0] + b" 12345678901234567890.1 .",
        lambda l: l.rsplit(b" ", 2)[0] + b" 1.5 .",
        lambda l: l.rsplit(b" ", 3)[0] + b" 7 0.1 .",
        lambda l: l.rsplit(b" ", 3)[0] + b" 000.000100 0.1 .",
        lambda l: l.replace(b'"-" ', b'"1.2.3.4, 5.6.7.8" ', 1),
        lambda l: l.replace(b" - - [", b" - user name [", 1),
        lambda l: l.replace(b" - - [", b" - \"q\" [", 1),
        lambda l: l.replace(b'" 200 ', b'" 200 -', 1),
        lambda l: b"::1" + l[l.index(b" "):],
        lambda l: b"-" + l[l.index(b" "):],
        lambda l: l,
    ]
    return rng.choice(ops)(line)


def test_nginx_config4_emulated(oracle, emu):
    paths = oracle.possible_paths(NGINX)
    o = oracle.Oracle(NGINX, paths)
    e = emu.Emu(NGINX, paths)
    assert e.status == 0, e.err
    lines = lpa.synth(lpa.SYNTH_NGINX, 20261017, 0, 4000).split(b"\n")[:-1]
    assert compare(o, e, lines, allow_fallback=False)["ok"] == 4000
    rng = random.Random(77)
    mut = [mutate_nginx(rng, l) for l in lines[:2000]] + [mutate(rng, l) for l in lines[2000:]]
    s = compare(o, e, mut)
    assert s["bad"] > 50 and s["ok"] > 500, s


def test_nginx_combined_format_emulated(oracle, emu):
    """The NGINX 'combined' log_format (hp/NginxHttpdLogFormatDissector.java:82-90)
    written out, on config-4 lines cut after the user agent."""
    lines = lpa.synth(lpa.SYNTH_NGINX, 5, 0, 300).split(b"\n")[:-1]
    ng = "$remote_addr - $remote_user [$time_local] \"$request\" $status $body_bytes_sent \"$http_referer\" \"$http_user_agent\""
    paths = oracle.possible_paths(ng)
    o = oracle.Oracle(ng, paths)
    e = emu.Emu(ng, paths)
    assert e.status == 0, e.err
    s = compare(o, e, [l.rsplit(b' "', 1)[0] for l in lines])
    assert s["ok"] > 250, s


STRF = lpa.SYNTH_FORMATS[lpa.SYNTH_STRFTIME]


def mutate_strf(rng, line):
    """Config-3 timestamp corners (StrfTimeToDateTimeFormatter + SMART resolver)."""
    i = line.index(b"[") + 1
    ts = line[i:i + 20]
    ops = [
        lambda t: t[:3] + b"APR" + t[6:],
        lambda t: t[:3] + b"sEp" + t[6:],
        lambda t: b"31/Apr" + t[6:],
        lambda t: b"29/Feb/2015" + t[11:],
        lambda t: b"29/Feb/2016" + t[11:],
        lambda t: t[:12] + b"24:00:00",
        lambda t: t[:12] + b"24:00:01",
        lambda t: t[:12] + b"23:60:00",
        lambda t: t[:12] + b"23:59:60",
        lambda t: b"32" + t[2:],
        lambda t: b"00" + t[2:],
        lambda t: t[:7] + b"0000" + t[11:],
        lambda t: t[:7] + b"0001" + t[11:],
        lambda t: t[:6] + b"-" + t[7:],
        lambda t: t[:11] + b":" + t[12:],
        lambda t: t[:2] + b"/Sept" + t[6:],
        lambda t: t,
    ]
    return line[:i] + rng.choice(ops)(ts) + line[i + 20:]


def test_strftime_config3_emulated(oracle, emu):
    paths = oracle.possible_paths(STRF)
    assert any(p.startswith("TIME.LOCALIZEDSTRING:") for p in paths)
    o = oracle.Oracle(STRF, paths)
    e = emu.Emu(STRF, paths)
    assert e.status == 0, e.err
    lines = lpa.synth(lpa.SYNTH_STRFTIME, 20261016, 0, 4000).split(b"\n")[:-1]
    s = compare(o, e, lines, allow_fallback=False)
    assert s["ok"] > 3700 and s["bad"] > 100, s  # 5 % malformed lines (BASELINE config 3)
    rng = random.Random(33)
    mut = [mutate_strf(rng, l) for l in lines[:2500] if b"[" in l and len(l) > 60] + [mutate(rng, l) for l in lines[2500:]]
    s = compare(o, e, mut)
    assert s["bad"] > 300 and s["ok"] > 1000, s


def test_multiline_sequence_emulated(oracle, emu, vectors):
    """HttpdLogFormatDissector sticky routing (hpt/MultiLineHttpdLogParserTest.java:64-124):
    one parser for the whole 12-line sequence."""
    seq = [c for c in vectors["cases"] if c["source"].startswith("hpt/MultiLineHttpdLogParserTest")]
    assert len(seq) == 12
    e = emu.Emu(seq[0]["logformat"], seq[0]["fields"])
    assert e.status == 0, e.err
    for c in seq:
        st, rec = e.parse(c["line"])
        assert golden_check.check_case(c, st, rec or {}) == [], c["source"]


MIXED = "combined\n" + NGINX + "\ncommon"


def mixed_lines(n, seed):
    """A mixed corpus (BASELINE config 5 shape): 'combined', NGINX config-4 and
    'common' lines, interleaved in runs."""
    rng = random.Random(seed)
    c2 = lpa.synth(lpa.SYNTH_COMBINED, seed, 0, n).split(b"\n")[:-1]
    c4 = lpa.synth(lpa.SYNTH_NGINX, seed, 0, n).split(b"\n")[:-1]
    out, i = [], 0
    while len(out) < n:
        k = rng.choice((0, 0, 1, 2))
        for _ in range(rng.randrange(1, 30)):
            if k == 0: out.append(c2[i % n])
            elif k == 1: out.append(c4[i % n])
            else: out.append(c2[i % n].rsplit(b' "', 2)[0])  # 'common': combined without referer / agent
            i += 1
    return out[:n]


def test_mixed_formats_emulated(oracle, emu):
    paths = oracle.possible_paths(MIXED)
    o = oracle.Oracle(MIXED, paths)
    e = emu.Emu(MIXED, paths)
    assert e.status == 0, e.err
    lines = mixed_lines(3000, 55)
    rng = random.Random(56)
    lines = [mutate(rng, l) if rng.random() < 0.1 else l for l in lines]
    s = compare(o, e, lines)
    assert s["ok"] > 2000 and s["bad"] > 20, s


HOSTS = ["a..b", "a-.b", "-a", "a.", "a.b.", "1a.b", "a.1b", "a1.b2", "a:80", "a.b:", "a.b:x", "a_b", "a!b", "a~b",
         "a'b", "a(b)", "a;b", "a=b", "a+b", "a$b", "a,b", "a*b", "a:1:2", "1.2.3.4", "1.2.3.4.5", "256.1.1.1",
         "01.2.3.4", "1.2.3", "1.2.3.4:99", "1.2.3.4x", "a.b.c-d.e", "a-b-c.d--e.f", "x.y.z.", "A.B.C:0",
         "a.b:2147483647", "a.b:2147483648", "a.b:00080", "9", "9.9", "9.a", "host-", "h.-x", ":80", "a%41b"]


def test_authority_variants_emulated(oracle, emu):
    """java.net.URI server authority parsing (parseServer / parseHostname /
    parseIPv4Address) on the referer URL's host part."""
    paths = all_paths(oracle)
    o = oracle.Oracle("combined", paths)
    e = emu.Emu("combined", paths)
    base = b'1.2.3.4 - - [01/Jan/2021:00:00:00 +0000] "GET / HTTP/1.1" 200 0 "http://%s/p?q=1" "u"'
    lines = []
    for h in HOSTS:
        for tail in ("", "/x", "#f", "?a"):
            lines.append(base.replace(b"%s/p?q=1", (h + tail + "/p?q=1").encode()))
    s = compare(o, e, lines)
    assert s["ok"] > 100, s


def test_synth_config5_mix():
    """lp_synth workload 5 (BASELINE config 5): per-line choice of 40 %
    'combined', 30 % NGINX config-4 and 30 % 'common' lines, deterministic per
    line index (any range re-generates bit-identically)."""
    lines = lpa.synth(lpa.SYNTH_MIXED, 20261018, 0, 20000).split(b"\n")[:-1]
    assert len(lines) == 20000
    nginx = sum(1 for l in lines if not l.endswith(b'"') and l[-1:] in (b"p", b"."))
    combined = sum(1 for l in lines if l.endswith(b'"'))
    common = len(lines) - nginx - combined
    assert abs(combined / 20000 - 0.4) < 0.02 and abs(nginx / 20000 - 0.3) < 0.02 and abs(common / 20000 - 0.3) < 0.02
    assert lpa.synth(lpa.SYNTH_MIXED, 20261018, 777, 5).split(b"\n")[:-1] == lines[777:782]


def test_mixed_config5_emulated(oracle, emu):
    """BASELINE config 5 corpus through the three-format handle: every line
    decided by its own (mutually exclusive) format, all paths, no FALLBACK."""
    fmt = lpa.SYNTH_FORMATS[lpa.SYNTH_MIXED]
    assert fmt == MIXED
    paths = oracle.possible_paths(fmt)
    o = oracle.Oracle(fmt, paths)
    e = emu.Emu(fmt, paths)
    assert e.status == 0, e.err
    lines = lpa.synth(lpa.SYNTH_MIXED, 20261018, 0, 3000).split(b"\n")[:-1]
    s = compare(o, e, lines, allow_fallback=False)
    assert s["ok"] == 3000, s


IP_TOKENS = ["api.jdoagd.com", "abc", "::1", "fe80::1", "1.2.3", "dead:beef", "-", "a:b", "1.2.3.4.5", "999.1.1.1",
             "cafe.babe", "x", "g", "a.b", "1.2.3.4", "01.2.3.4", "ab:cd:ef", "1::", ":", "a-b", "--", "a.-"]


@pytest.mark.parametrize("fmt", ["nginx", "common", "mixed"])
def test_ip_token_variants_emulated(oracle, emu, fmt):
    """FORMAT_IP / FORMAT_CLF_IP (TokenParser.java:43-52) on non-IPv4 hosts:
    a host whose IPv6-branch ends cannot be followed by the format's next
    literal is decided (BAD or the next format), the rest is exact or FALLBACK."""
    f = {"nginx": NGINX, "common": "common", "mixed": MIXED}[fmt]
    paths = oracle.possible_paths(f)
    o = oracle.Oracle(f, paths)
    e = emu.Emu(f, paths)
    base = lpa.synth(lpa.SYNTH_MIXED, 20261018, 0, 60).split(b"\n")[:-1]
    lines = [t.encode() + b" " + l.split(b" ", 1)[1] for l in base for t in IP_TOKENS[:: 1 + len(l) % 3]]
    s = compare(o, e, lines)
    assert s["fallback"] < len(lines) // 4, s


def test_setup_vectors_planner(emu, vectors):
    """The device planner (plan.cpp, the code lp_compile runs) refuses the
    same requests as the reference: MissingDissectorsException with the path."""
    for c in vectors["setup_cases"]:
        with pytest.raises(RuntimeError) as ei:
            emu.Emu(c["logformat"], c["fields"])
        assert "failed -2" in str(ei.value) and c["message_contains"] in str(ei.value), c["source"]


def test_utf8_user_agents_emulated(oracle, emu):
    """UTF-8 user agents / users stay on the device path with exact records;
    UTF-8 in URIs, U+0085/U+2028/U+2029 and invalid sequences go to FALLBACK"""
    import corpora
    base = lpa.synth_combined(20261016, 0, 1500).split(b"\n")[:-1]
    o = oracle.Oracle("combined", all_paths(oracle))
    e = emu.Emu("combined", all_paths(oracle))
    s = compare(o, e, corpora.utf8_ua_lines(base, 5), allow_fallback=False)
    assert s["ok"] == 1500, s
    hard = corpora.utf8_hard_lines(base, 6)
    s = compare(o, e, hard)
    assert s["fallback"] > 500 and s["ok"] > 200, s
    # NGINX: CLF_IP tokens (the IPv6 '.' consumes one char, not one byte)
    paths = oracle.possible_paths(NGINX)
    o = oracle.Oracle(NGINX, paths)
    e = emu.Emu(NGINX, paths)
    lines = lpa.synth(lpa.SYNTH_NGINX, 20261018, 0, 800).split(b"\n")[:-1]
    rng = random.Random(3)
    u8 = []
    for l in lines:
        i = l.index(b" - ")
        u8.append(l[:i] + b" - " + rng.choice(corpora.USERS).encode() + l[l.index(b" ", i + 3):])
    s = compare(o, e, u8)
    assert s["ok"] > 700, s
    compare(o, e, [b"1:2\xc3\xa9 - - [" + l.split(b"[", 1)[1] for l in lines[:50]])


def upstream_lines(n, seed):
    """NGINX lines with $upstream_addr / $upstream_status lists ([^\\s]* items),
    quoted and unquoted, and $binary_remote_addr"""
    rng = random.Random(seed)
    out = []
    for _ in range(n):
        k = rng.choice([1, 1, 1, 2, 3])
        addrs = [rng.choice(["10.0.%d.%d:80" % (rng.randrange(256), rng.randrange(256)), "unix:/tmp/sock",
                             "backend_%d" % rng.randrange(9), "[::1]:8080"]) for _ in range(k)]
        st = [str(rng.choice([200, 502, 504, 404])) for _ in range(k)]
        sep = [rng.choice([", ", ", ", " : "]) for _ in range(k - 1)]
        addr = addrs[0] + "".join(s + a for s, a in zip(sep, addrs[1:]))
        stat = st[0] + "".join(s + a for s, a in zip(sep, st[1:]))
        ip = "".join("\\x%02X" % rng.randrange(256) for _ in range(4))
        if rng.random() < 0.1:
            addr = addr.replace(", ", ", : ", 1)  # a server piece the reference cannot split
        out.append(('%s "%s" %s %s "GET /x HTTP/1.1"' % (rng.choice(["1.2.3.4", "-"]), addr, stat, ip)).encode())
    return out


UPSTREAM_FMT = '$remote_addr "$upstream_addr" $upstream_status $binary_remote_addr "$request"'


def test_upstream_lists_and_binary_ip_emulated(oracle, emu):
    """UpstreamModule [^\\s]* lists (UpstreamListDissector split) and
    BinaryIPDissector (signed bytes) on the device"""
    paths = oracle.possible_paths(UPSTREAM_FMT)
    o = oracle.Oracle(UPSTREAM_FMT, paths)
    e = emu.Emu(UPSTREAM_FMT, paths)
    assert e.status == 0, e.err
    s = compare(o, e, upstream_lines(3000, 5))
    assert s["ok"] > 1500, s
    st, rec = e.parse(b'- "a:1, b:2 : c:3" 504 \\xC0\\xA8\\x01\\xFF "GET / HTTP/1.1"')
    assert st == 0
    assert "-64.-88.1.-1" in rec["IP:connection.client.host"]  # ($remote_addr "-" adds a null)
    assert rec["UPSTREAM_ADDR:nginxmodule.upstream.addr.1.redirected"] == ["c:3"]


CACHE_FMT = '$remote_addr $upstream_cache_status [$time_local] "$request" $status'


def cache_status_lines(n, seed):
    """$upstream_cache_status: the seven words of UpstreamModule's alternation
    plus near misses (BAD lines)"""
    rng = random.Random(seed)
    words = ["MISS", "BYPASS", "EXPIRED", "STALE", "UPDATING", "REVALIDATED", "HIT",
             "MISSING", "HITS", "-", "miss", "", "REVALIDATE", "STALE STALE"]
    out = []
    for i in range(n):
        w = rng.choice(words[:7]) if rng.random() < 0.8 else rng.choice(words[7:])
        out.append(('10.1.%d.%d %s [%02d/Mar/2024:10:%02d:%02d +0100] "GET /p?x=%d HTTP/1.1" %d' % (
            rng.randrange(256), rng.randrange(256), w, 1 + i % 28, i % 60, (i * 7) % 60, i,
            rng.choice([200, 304, 404]))).encode())
    return out


def test_upstream_cache_status_emulated(oracle, emu):
    """$upstream_cache_status (?:MISS|BYPASS|...|HIT) on the device"""
    paths = oracle.possible_paths(CACHE_FMT)
    o = oracle.Oracle(CACHE_FMT, paths)
    e = emu.Emu(CACHE_FMT, paths)
    assert e.status == 0, e.err
    s = compare(o, e, cache_status_lines(3000, 8))
    assert s["ok"] > 2000 and s["bad"] > 300 and s["fallback"] == 0, s


COOKIE_FMT = '%h %l %u %t "%r" %>s %b "%{Cookie}i"'


def cookie_lines(n, seed):
    """'combined'-like lines with a request Cookie header: upper-case names,
    blanks around names and values, empty pieces, names without '=',
    %XX / '+' values, and a few invalid escapes / non-ASCII bytes (FALLBACK)"""
    rng = random.Random(seed)
    base = lpa.synth_combined(seed, 0, n).split(b"\n")[:-1]
    out = []
    for l in base:
        head = l.rsplit(b' "', 2)[0]
        pieces = []
        for _ in range(rng.randrange(0, 7)):
            name = rng.choice(["session", "JSESSIONID", "_ga", "Theme", "a b", " pad", "x-Y_z", ""])
            val = rng.choice(["abc", "1234", "%41%42", "a+b", "%C3%A9t%C3%A9", " spaced ", "", "x=y", "%7E%2F"])
            form = rng.random()
            pieces.append(name if form < 0.15 else name + "=" + val)
        hdr = "; ".join(pieces) + ("; " if rng.random() < 0.2 else "")
        if rng.random() < 0.05:
            hdr += "; bad=%zz"
        if rng.random() < 0.03:
            hdr += "; u=é"
        out.append(head + b' "' + hdr.encode() + b'"')
    return out


@pytest.mark.parametrize("fields", [["HTTP.COOKIE:request.cookies.*"],
                                    ["HTTP.COOKIE:request.cookies.session", "HTTP.COOKIE:request.cookies.theme",
                                     "HTTP.COOKIES:request.cookies", "STRING:request.status.last"]])
def test_request_cookies_emulated(oracle, emu, fields):
    """RequestCookieListDissector: split / trim / lower-case / resilientUrlDecode"""
    o = oracle.Oracle(COOKIE_FMT, fields)
    e = emu.Emu(COOKIE_FMT, fields)
    assert e.status == 0, e.err
    s = compare(o, e, cookie_lines(3000, 11))
    assert s["ok"] > 2500 and s["fallback"] < 300, s


QS_FMT = '%h %l %u %t "%r" %>s %b "%q"'


def querystring_lines(n, seed):
    """lines with a raw %q query string token: '?'-prefixed or empty, upper-case
    names, empty pieces, %XX / '+' values, a few invalid escapes (FALLBACK)"""
    rng = random.Random(seed)
    base = lpa.synth_combined(seed, 0, n).split(b"\n")[:-1]
    out = []
    for l in base:
        head = l.rsplit(b' "', 2)[0]
        pieces = []
        for _ in range(rng.randrange(0, 6)):
            name = rng.choice(["aap", "Res", "q", "", "x%41", "utm_source"])
            val = rng.choice(["noot", "1024x768", "%41%42", "a+b", "%C3%A9", "", "x=y"])
            pieces.append(name if rng.random() < 0.15 else name + "=" + val)
        q = "&".join(pieces) + ("&" if rng.random() < 0.2 else "")
        if q and rng.random() < 0.7:
            q = "?" + q
        if rng.random() < 0.04:
            q += "&bad=%g1"
        out.append(head + b' "' + q.encode() + b'"')
    return out


@pytest.mark.parametrize("fields", [["STRING:request.querystring.*"],
                                    ["STRING:request.querystring.aap", "STRING:request.querystring.res",
                                     "HTTP.QUERYSTRING:request.querystring"]])
def test_querystring_token_emulated(oracle, emu, fields):
    """QueryStringFieldDissector on a raw %q token"""
    o = oracle.Oracle(QS_FMT, fields)
    e = emu.Emu(QS_FMT, fields)
    assert e.status == 0, e.err
    s = compare(o, e, querystring_lines(3000, 13))
    assert s["ok"] > 2600 and s["fallback"] < 250, s


ISO_FMT = '$remote_addr - - [$time_iso8601] "$request" $status'


def iso_lines(n, seed):
    """NGINX $time_iso8601 lines: valid stamps and the resolver corners
    (day clamp, 24:00:00, offsets up to +-18:00, invalid month / day /
    offset / sign -> BAD)"""
    rng = random.Random(seed)
    out = []
    for _ in range(n):
        y = rng.choice([2000, 2012, 2015, 2016, 2019, 2024, 1999, 9999, 1000])
        mo = rng.choice(list(range(1, 13)) + [0, 13])
        d = rng.choice(list(range(1, 29)) + [29, 30, 31, 0, 32])
        h = rng.choice(list(range(0, 24)) + [24])
        mi = rng.choice([0, 1, 30, 59, 60])
        s = rng.choice([0, 5, 59, 60])
        sign = rng.choice("++--|")
        oh, om = rng.choice([(0, 0), (1, 0), (5, 30), (14, 0), (18, 0), (19, 0), (2, 60)])
        if rng.random() < 0.7:  # mostly valid
            mo, d, h, mi, s, oh, om, sign = rng.randrange(1, 13), rng.randrange(1, 29), rng.randrange(24), \
                rng.randrange(60), rng.randrange(60), rng.randrange(15), rng.choice([0, 30, 45]), rng.choice("+-")
        ts = "%04d-%02d-%02dT%02d:%02d:%02d%s%02d:%02d" % (y, mo, d, h, mi, s, sign, oh, om)
        out.append(('10.0.0.%d - - [%s] "GET /x?a=%d HTTP/1.1" 200' % (rng.randrange(256), ts, rng.randrange(99))).encode())
    return out


def test_iso8601_timestamps_emulated(oracle, emu):
    """TimeStampDissector("TIME.ISO8601", "yyyy-MM-dd'T'HH:mm:ssXXX") on the device"""
    paths = oracle.possible_paths(ISO_FMT)
    o = oracle.Oracle(ISO_FMT, paths)
    e = emu.Emu(ISO_FMT, paths)
    assert e.status == 0, e.err
    s = compare(o, e, iso_lines(4000, 21), allow_fallback=False)
    assert s["ok"] > 2500 and s["bad"] > 300, s


SETCOOKIE_FMT = '%h %l %u %t "%r" %>s %b "%{Set-Cookie}o"'
_DAYS = ["Mon", "Tue", "Wed", "Thu", "Fri", "Sat", "Sun"]
_MONS = ["Jan", "Feb", "Mar", "Apr", "May", "Jun", "Jul", "Aug", "Sep", "Oct", "Nov", "Dec"]


def _expires(rng):
    """an "expires" date: mostly "EEE, dd-MMM-yyyy HH:mm:ss GMT" with the right
    day name; some with a wrong day name, another zone or another layout
    (the reference throws on those: FALLBACK)"""
    import datetime
    d = datetime.datetime(1990, 1, 1) + datetime.timedelta(seconds=rng.randrange(0, 60 * 365 * 86400))
    day = _DAYS[d.weekday()]
    r = rng.random()
    if r < 0.05:
        day = _DAYS[(d.weekday() + 1) % 7]
    zone = "GMT" if rng.random() > 0.05 else rng.choice(["UTC", "PST", "CET"])
    if rng.random() < 0.04:
        return "%s, %02d %s %04d %02d:%02d:%02d %s" % (day, d.day, _MONS[d.month - 1], d.year, d.hour, d.minute,
                                                       d.second, zone)
    return "%s, %02d-%s-%04d %02d:%02d:%02d %s" % (day, d.day, _MONS[d.month - 1], d.year, d.hour, d.minute,
                                                   d.second, zone)


def setcookie_lines(n, seed):
    """'combined'-like lines ending in a Set-Cookie header list: several
    cookies joined by ", " with expires / path / domain / comment / Secure /
    HttpOnly attributes, upper-case and blank-padded names, "-" and empty
    headers, and inputs outside the restated subset or on which the reference
    throws (Max-Age, quotes, '$' names, reserved names, names without '=',
    bad dates: FALLBACK)"""
    rng = random.Random(seed)
    base = lpa.synth_combined(seed, 0, n).split(b"\n")[:-1]
    out = []
    for l in base:
        head = l.rsplit(b' "', 2)[0]
        r = rng.random()
        if r < 0.15:
            hdr = "-"
        elif r < 0.18:
            hdr = ""
        else:
            cookies = []
            for _ in range(rng.randrange(1, 5)):
                name = rng.choice(["SESSION", "sid", "NBA-1", "_ga", " pad ", "x.y", "Theme", "sid"])
                if rng.random() < 0.08:
                    name = rng.choice(["a b", "$v", "Path", "", "x,z"])
                val = rng.choice(["1234", "", "abc=def", "a:b", "bla bla", "%41", "x,y", "1234"])
                if rng.random() < 0.03:
                    val = 'q"q'

                c = name + "=" + val if rng.random() > 0.03 else name
                for _ in range(rng.randrange(0, 4)):
                    a = rng.random()
                    if a < 0.35:
                        c += "; expires=" + _expires(rng)
                    elif a < 0.5:
                        c += "; path=/" + rng.choice(["", "xx", "a/b"])
                    elif a < 0.62:
                        c += "; domain=." + rng.choice(["basj.es", "example.com"])
                    elif a < 0.7:
                        c += "; comment=bla bla"
                    elif a < 0.78:
                        c += "; " + rng.choice(["Secure", "HttpOnly", "secure"])
                    elif a < 0.85:
                        c += "; Expires=" + _expires(rng)
                    elif a < 0.865:
                        c += "; Max-Age=" + rng.choice(["10", "x"])
                    elif a < 0.9:
                        c += ";;  path = /sp "
                    else:
                        c += "; Domain=.Basj.ES"
                cookies.append(c)
            hdr = ", ".join(cookies) + (", " if rng.random() < 0.05 else "")
        out.append(head + b' "' + hdr.encode() + b'"')
    return out


SETCOOKIE_FIELDS = [
    ["HTTP.SETCOOKIES:response.cookies", "HTTP.SETCOOKIE:response.cookies.*"],
    ["HTTP.SETCOOKIE:response.cookies.sid", "STRING:response.cookies.sid.value", "STRING:response.cookies.sid.expires",
     "TIME.EPOCH:response.cookies.sid.expires", "STRING:response.cookies.sid.path",
     "STRING:response.cookies.sid.domain", "STRING:response.cookies.sid.comment",
     "STRING:response.cookies.session.value", "TIME.EPOCH:response.cookies.nba-1.expires",
     "STRING:request.status.last"],
]


@pytest.mark.parametrize("which", [0, 1])
def test_set_cookies_emulated(oracle, emu, which):
    """ResponseSetCookieListDissector + ResponseSetCookieDissector: ", " split
    with the expires join, HttpCookie names, "; " attributes, expires dates"""
    fields = SETCOOKIE_FIELDS[which]
    o = oracle.Oracle(SETCOOKIE_FMT, fields)
    e = emu.Emu(SETCOOKIE_FMT, fields)
    assert e.status == 0, e.err
    s = compare(o, e, setcookie_lines(3000, 21 + which))
    assert s["ok"] > 1000 and s["fallback"] < 2000, s


def test_strftime_conversions_emulated(oracle, emu):
    """Every strftime conversion the reference converts (strf_corpus): the
    device code's parse + SMART resolution against the oracle's, on printed
    and mutated values; only the stray non-ASCII letters stay FALLBACK.
    A variable-width number directly followed by another (JDK adjacent
    value parsing) keeps the handle off the device, as the oracle refuses it."""
    import strf_corpus
    tot = {"ok": 0, "bad": 0, "fallback": 0}
    for fmt, lines in strf_corpus.corpus(20261017, per_pattern=120):
        o = oracle.Oracle(fmt, strf_corpus.FIELDS)
        e = emu.Emu(fmt, strf_corpus.FIELDS)
        s = compare(o, e, lines)
        for k in tot:
            tot[k] += s[k]
        assert s["fallback"] <= len(lines) // 10, (fmt, s)
    assert tot["ok"] > 800 and tot["bad"] > 150, tot
    e = emu.Emu('%h [%{%k%M}t]', strf_corpus.FIELDS)
    assert e.status == -3  # LP_E_UNSUPPORTED


def test_type_remapping_emulated(oracle, emu):
    """Type remappings (core/Parser.java:636-677, Parsable.java:160-176): URLs
    in query parameters / the user agent remapped to HTTP.URI, dissected by the
    derived URI stages; exact against the oracle's restatement."""
    import remap_corpus as rc
    lines = rc.corpus(7, 1500)
    o = oracle.Oracle(rc.FORMAT, rc.FIELDS, rc.REMAPS)
    e = emu.Emu(rc.FORMAT, rc.FIELDS, rc.REMAPS)
    assert e.status == 0, e.err
    s = compare(o, e, lines)
    assert s["ok"] > 750 and s["fallback"] < 0.4 * len(lines), s


def test_type_remapping_same_type_planner(oracle, emu):
    """A remapping to the value's own type is a DissectionFailure for every
    line that delivers the value (core/Parsable.java:163-168): the oracle says
    BAD for those lines; the planner leaves the program to FALLBACK."""
    fields = ["STRING:request.firstline.uri.query.a", "HTTP.PATH:request.firstline.uri.path"]
    rm = [("request.firstline.uri.query.a", "STRING")]
    o = oracle.Oracle("combined", fields, rm)
    e = emu.Emu("combined", fields, rm)
    assert e.status == -3 and "own type" in e.err, e.err
    base = '1.2.3.4 - - [10/Oct/2020:13:55:36 +0200] "GET %s HTTP/1.1" 200 5 "-" "x"'
    assert o.parse(base % "/p?a=1")[0] == oracle.BAD
    assert o.parse(base % "/p?b=1")[0] == oracle.OK
    assert e.parse(base % "/p?b=1")[0] == 2



def test_strftime_fixed_plan_edges_emulated(emu):
    """strf_fixed (the fixed-layout plan: all literals and digit positions
    checked at once with byte masks, fields at fixed offsets) decides every
    value exactly as the general element loop: valid values at every byte
    offset of a word, every single-byte mutation of them (digits, letters in
    both cases, separators, non-ASCII), wrong widths, offsets "+0000" /
    "-0000" / out-of-range, and a layout with a field given twice (no plan:
    the general loop's "must agree" check)."""
    import random
    import strf_corpus
    rng = random.Random(20261018)
    cases = [("%d/%b/%Y %T", True), ("%a, %d %b %Y %T %z", True), ("%D %r", True), ("%Y-%j %H:%M", True),
             ("%d/%b/%Y %I:%M %P", True), ("%F %T.msec_frac %z", True), ("%F %R:%S.usec_frac", True),
             ("%d/%b/%Y %T %d", False), ("%a %A", False)]
    alphabet = b"0123456789aAbBzZ:/ .,+-\x80\xc3"
    n_vals = 0
    for pat, plan in cases:
        e = emu.Emu('%h [%{' + pat + '}t] "%r"', strf_corpus.FIELDS)
        assert e.status == 0, (pat, e.err)
        vals = []
        for _ in range(40):
            dt = strf_corpus.datetime.datetime(1971, 1, 1) + strf_corpus.datetime.timedelta(
                seconds=rng.randrange(0, 60 * 365 * 86400), microseconds=rng.randrange(1000000))
            v = strf_corpus.render(pat, dt, rng.choice([0, -300, 330, 60 * 14]))
            vals.append(v.encode())
        v0 = vals[0]
        for i in range(len(v0)):  # every position, several replacement bytes
            for c in rng.sample(alphabet, 6):
                vals.append(v0[:i] + bytes([c]) + v0[i + 1:])
        vals += [v0[:-1], v0 + b"0", v0.upper(), v0.lower(), b""]
        if b"+" in v0 or b"-" in v0[-5:]:
            k = len(v0) - 5
            vals += [v0[:k] + z for z in (b"+0000", b"-0000", b"+1860", b"-0960", b"+2400", b"|0100", b"+0a00")]
        for v in vals:
            for off in range(4):
                nf, fixed = e.strf(v, off, True)
                _, general = e.strf(v, off, False)
                assert (nf > 0) == plan, (pat, nf)
                assert fixed == general, (pat, v, off, fixed, general)
                n_vals += 1
    assert n_vals > 3000


def test_upstream_list_register_scan_emulated(emu):
    """uplist_at_r (the first-leaf candidate of NGINX upstream lists from
    32 bytes in registers, bit masks for digits / '.' / ',' / ':' / ' ')
    returns what uplist_at (one read per byte) returns: lists of 1-4 items
    with ", " and " : " separators, space runs, separators without the
    space or at the end, 19-digit runs, lists ending at the line end or
    continuing, lists reaching byte 31, 32, 33 and beyond the registers,
    at every byte offset of a word."""
    import random
    rng = random.Random(20261018)

    def item(dec):
        a = "".join(rng.choice("0123456789") for _ in range(rng.choice([1, 1, 2, 3, 19, 20])))
        if not dec or rng.random() < 0.1:
            return a
        return a + "." + "".join(rng.choice("0123456789") for _ in range(rng.choice([0, 1, 3, 3, 19])))
    seps = [", ", " : ", ",", ":", " , ", ",  ", " ", ", ,", ": ", "-", ""]
    n = 0
    for _ in range(6000):
        dec = rng.random() < 0.7
        k = rng.choice([1, 1, 2, 3, 4, 6])
        s = item(dec)
        for _ in range(k - 1):
            s += rng.choice(seps[:2] * 4 + seps) + item(dec)
        if rng.random() < 0.3:
            s += rng.choice(seps)
        pre = rng.choice(["", "x ", "12 ", "- - [a] "])
        post = rng.choice(["", " ", " .", " p", "\" 200", " " * rng.randint(0, 40) + "x"])
        line = (pre + s + post).encode()
        p = len(pre)
        for off in range(4):
            a, b = emu.uplist(line, p, off, dec)
            assert a == b, (line, p, off, dec, a, b)
            n += 1
    # every length around the register window
    for L in range(28, 40):
        for dec in (True, False):
            body = ("0.1, " * 10)[:L] if dec else ("1, " * 16)[:L]
            for post in ("", " p"):
                line = (body + post).encode()
                for off in range(4):
                    a, b = emu.uplist(line, 0, off, dec)
                    assert a == b, (line, off, dec, a, b)
                    n += 1
    assert n > 20000


def test_upstream_list_split_register_edges_emulated(emu):
    """uplist_items_r / secms_value_r (the URI kernel's list stage on a token
    of at most 32 bytes held in registers) against uplist_items /
    secms_value (one read per byte) on constructed edge tokens: lengths 31,
    32 and 33 (33: not loaded, the byte path alone), a ', ' or ': ' separator
    in the last two bytes, separators only, whitespace-only tokens, empty
    servers, ': ' pairs without parts, at every byte offset of a word."""
    import random
    rng = random.Random(20261019)
    toks = [b"", b" ", b"   ", b"\t \t", b", ", b", , ", b": ", b" : ", b",", b":", b"1, ", b"1: ", b"1, 2: ",
            b", 1", b": 1", b"1 : 2", b"1,2", b"1:2", b"0.001, 0.002 : 0.003", b"1.5, -, 2.25"]
    # lengths around the register window, the separator placed at its end
    for L in (30, 31, 32, 33, 34):
        for tail in (b", ", b": ", b",", b" ", b", 7", b": 7", b""):
            body = b"0.1, 2.25 : 3.0, " * 4
            t = body[: max(0, L - len(tail))] + tail
            toks.append(t[:L])
            toks.append((b" " * L)[:L])
            toks.append((b", " * 20)[:L])
            toks.append((b": " * 20)[:L])
    for _ in range(3000):
        n = rng.choice([rng.randint(0, 34), 31, 32, 33])
        alpha = rng.choice([b"0123456789., :", b"0123456789., : \t", b"ab.1, :-"])
        toks.append(bytes(rng.choice(alpha) for _ in range(n)))
    n_reg = 0
    for t in toks:
        dec = all(c in b"0123456789." for c in t.replace(b", ", b"").replace(b": ", b"").replace(b" ", b""))
        for off in range(4):
            (nb, ib), (nr, ir) = emu.uplist_items(t, off, dec)
            if len(t) > 32:
                assert nr == -2, (t, nr)
                continue
            n_reg += 1
            assert nr == nb, (t, off, nb, nr)
            if dec:
                assert ir == ib, (t, off, ib, ir)
            else:
                assert [x[:4] for x in ir] == [x[:4] for x in ib], (t, off, ib, ir)
    assert n_reg > 5000
