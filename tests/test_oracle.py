"""The oracle (CPU restatement, oracle/) pinned against the reference's own
test vectors (tests/golden/reference_vectors.json, transcribed from the
reference JUnit tests) and the reference's demo log (config 1)."""
import pytest

import golden_check

# the regex TokenFormatDissector.prepareForRun builds for
# 'combined' with every output requested
COMBINED_REGEX = (
    r'^([^\s]*)\Q \E([0-9]+|-)\Q \E([^\s]*)\Q [\E([0-3][0-9]/(?:[a-zA-Z][a-zA-Z][a-zA-Z])/[1-9][0-9][0-9][0-9]'
    r':[0-9][0-9]:[0-9][0-9]:[0-9][0-9] [\+|\-][0-9][0-9][0-9][0-9])\Q] "\E(.*)\Q" \E([^\s]*)\Q \E([0-9]+|-)'
    r'\Q "\E(.*?)\Q" "\E(.*?)\Q"\E$')


def test_possible_paths_combined(oracle):
    paths = oracle.possible_paths("combined")
    assert len(paths) == 123
    assert "TIME.EPOCH:request.receive.time.epoch" in paths
    assert "STRING:request.firstline.uri.query.*" in paths
    assert "TIME.ZONE:request.receive.time.timezone" in paths


def test_possible_paths_reference_test(oracle):
    # hpt/ApacheHttpdLogParserTest.java:283-294 (maxDepth 5)
    fmt = ("%%%h %a %A %l %u %t \"%r\" %>s %b %p \"%q\" \"%!200,304,302{Referer}i\" %D "
           "\"%200{User-agent}i\" \"%{Cookie}i\" \"%{Set-Cookie}o\" \"%{If-None-Match}i\" \"%{Etag}o\"")
    paths = oracle.possible_paths(fmt, 5)
    assert "TIME.SECOND:request.receive.time.second" in paths
    assert "STRING:request.firstline.uri.query.*" in paths
    assert "STRING:response.cookies.*.expires" in paths
    assert "HTTP.HEADER:response.header.etag" in paths
    assert "FIXED_STRING:fixed_string" not in paths


def test_regex_combined(oracle):
    o = oracle.Oracle("combined", oracle.possible_paths("combined"))
    assert o.regex() == COMBINED_REGEX


@pytest.mark.parametrize("idx", range(len(__import__("golden_check").load_vectors()["cases"])))
def test_golden_vector(oracle, vectors, idx):
    cases = vectors["cases"]
    if idx >= len(cases):
        pytest.skip("no such case")
    c = cases[idx]
    if c["source"].startswith("hpt/MultiLineHttpdLogParserTest"):
        pytest.skip("sequence case: covered by test_multiline_sequence")
    o = oracle.Oracle(c["logformat"], c["fields"], c["remaps"])
    st, rec = o.parse(c["line"])
    assert golden_check.check_case(c, st, rec or {}) == [], c["source"]


def test_multiline_sequence(oracle, vectors):
    seq = [c for c in vectors["cases"] if c["source"].startswith("hpt/MultiLineHttpdLogParserTest")]
    assert len(seq) == 12
    o = oracle.Oracle(seq[0]["logformat"], seq[0]["fields"])  # one stateful parser (sticky format)
    for c in seq:
        st, rec = o.parse(c["line"])
        assert golden_check.check_case(c, st, rec or {}) == [], c["source"]


def test_url_decode_vectors(oracle, vectors):
    for inp, want in vectors["url_decode"]["vectors"]:
        assert oracle.resilient_url_decode(inp) == want, inp


def test_demolog_all_match(oracle, demolog_lines):
    # config 1: examples/demolog/hackers-access.log, every line parses
    o = oracle.Oracle("combined", oracle.possible_paths("combined"))
    assert len(demolog_lines) == 3456
    bad = [l for l in demolog_lines if o.parse_raw(l)[0] != oracle.OK]
    assert bad == []


def test_bad_lines(oracle):
    o = oracle.Oracle("combined", ["IP:connection.client.host", "TIME.EPOCH:request.receive.time.epoch"])
    good = b'1.2.3.4 - - [31/Dec/2012:23:00:44 -0700] "GET / HTTP/1.1" 200 12 "-" "ua"'
    assert o.parse_raw(good)[0] == oracle.OK
    assert o.parse_raw(good.replace(b"Dec", b"Foo"))[0] == oracle.BAD        # DateTimeParseException
    assert o.parse_raw(good.replace(b"31/Dec", b"00/Dec"))[0] == oracle.BAD  # day 0
    assert o.parse_raw(good.replace(b" 12 ", b" x12 "))[0] == oracle.BAD     # %b not a number
    assert o.parse_raw(good[:-1])[0] == oracle.BAD                           # missing closing quote
    # SMART resolver: 31/Apr -> 30/Apr (JDK 8 IsoChronology.resolveYMD)
    st, rec = oracle.Oracle("combined", ["TIME.DAY:request.receive.time.day"]).parse(
        good.replace(b"31/Dec/2012", b"31/Apr/2012"))
    assert st == oracle.OK and rec["TIME.DAY:request.receive.time.day"] == [{"l": 30}]


# hpt/NginxLogFormatTest.java:95-204 (testCompareApacheAndNginxOutput): the NGINX
# 'combined' and the Apache combined-without-logname formats deliver the same
# values for the same line
NGINX_VS_APACHE_FIELDS = [
    "HTTP.URI:request.referer", "HTTP.PROTOCOL:request.referer.protocol", "HTTP.USERINFO:request.referer.userinfo",
    "HTTP.HOST:request.referer.host", "HTTP.PORT:request.referer.port", "HTTP.PATH:request.referer.path",
    "HTTP.QUERYSTRING:request.referer.query", "STRING:request.referer.query.*", "HTTP.REF:request.referer.ref",
    "TIME.STAMP:request.receive.time", "TIME.DAY:request.receive.time.day",
    "TIME.MONTHNAME:request.receive.time.monthname", "TIME.MONTH:request.receive.time.month",
    "TIME.WEEK:request.receive.time.weekofweekyear", "TIME.YEAR:request.receive.time.weekyear",
    "TIME.YEAR:request.receive.time.year", "TIME.HOUR:request.receive.time.hour",
    "TIME.MINUTE:request.receive.time.minute", "TIME.SECOND:request.receive.time.second",
    "TIME.MILLISECOND:request.receive.time.millisecond", "TIME.DATE:request.receive.time.date",
    "TIME.TIME:request.receive.time.time", "TIME.ZONE:request.receive.time.timezone",
    "TIME.EPOCH:request.receive.time.epoch", "TIME.DAY:request.receive.time.day_utc",
    "TIME.MONTHNAME:request.receive.time.monthname_utc", "TIME.MONTH:request.receive.time.month_utc",
    "TIME.WEEK:request.receive.time.weekofweekyear_utc", "TIME.YEAR:request.receive.time.weekyear_utc",
    "TIME.YEAR:request.receive.time.year_utc", "TIME.HOUR:request.receive.time.hour_utc",
    "TIME.MINUTE:request.receive.time.minute_utc", "TIME.SECOND:request.receive.time.second_utc",
    "TIME.MILLISECOND:request.receive.time.millisecond_utc", "TIME.DATE:request.receive.time.date_utc",
    "TIME.TIME:request.receive.time.time_utc", "BYTESCLF:response.body.bytes", "BYTES:response.body.bytes",
    "STRING:request.status.last", "HTTP.USERAGENT:request.user-agent", "HTTP.FIRSTLINE:request.firstline",
    "HTTP.METHOD:request.firstline.method", "HTTP.URI:request.firstline.uri",
    "HTTP.PROTOCOL:request.firstline.uri.protocol", "HTTP.USERINFO:request.firstline.uri.userinfo",
    "HTTP.HOST:request.firstline.uri.host", "HTTP.PORT:request.firstline.uri.port",
    "HTTP.PATH:request.firstline.uri.path", "HTTP.QUERYSTRING:request.firstline.uri.query",
    "STRING:request.firstline.uri.query.*", "HTTP.REF:request.firstline.uri.ref",
    "HTTP.PROTOCOL_VERSION:request.firstline.protocol", "HTTP.PROTOCOL:request.firstline.protocol",
    "HTTP.PROTOCOL.VERSION:request.firstline.protocol.version", "IP:connection.client.host"]


def test_nginx_equals_apache(oracle):
    nginx = ("$remote_addr - $remote_user [$time_local] \"$request\" $status $body_bytes_sent \"$http_referer\" "
             "\"$http_user_agent\"")
    apache = "%h - %u %t \"%r\" %>s %b \"%{Referer}i\" \"%{User-Agent}i\""
    line = ("1.2.3.4 - - [23/Aug/2010:03:50:59 +0000] \"POST /foo.html?aap&noot=mies HTTP/1.1\" 200 2 "
            "\"http://www.example.com/bar.html?wim&zus=jet\" \"Niels Basjes/1.0\"")
    fields = []
    for f in NGINX_VS_APACHE_FIELDS:
        if f.endswith(".*"):
            fields += [f[:-1] + p for p in ("aap", "noot", "mies", "wim", "zus", "jet")]
        else:
            fields.append(f)
    sa, ra = oracle.Oracle(apache, fields).parse(line)
    sn, rn = oracle.Oracle(nginx, fields).parse(line)
    assert sa == sn == 0

    def as_str(vals):  # TestRecord.setStringValue: Value.getString of each delivered value
        return [v if not isinstance(v, dict) else (None if v["l"] is None else str(v["l"])) for v in vals]
    for f in fields:
        assert (f in ra) == (f in rn), f
        if f in ra:
            assert as_str(ra[f]) == as_str(rn[f]), f


def test_setup_vectors_oracle(oracle, vectors):
    """Setup-time failures transcribed from the reference (MissingDissectorsException)."""
    assert len(vectors["setup_cases"]) >= 3
    for c in vectors["setup_cases"]:
        with pytest.raises(Exception) as ei:
            oracle.Oracle(c["logformat"], c["fields"])
        assert c["error"] in str(ei.value) and c["message_contains"] in str(ei.value), c["source"]


def _fnv1a(b):
    h = 1469598103934665603
    for c in b:
        h = ((h ^ c) * 1099511628211) & 0xFFFFFFFFFFFFFFFF
    return h


def test_digest_lines_matches_records(oracle):
    """orc_digest_lines (the whole-batch parity helper) gives each line's
    status and the FNV-1a of the same record orc_parse writes."""
    fields = oracle.possible_paths("combined")
    lines = [b'1.2.3.4 - - [10/Oct/2000:13:55:36 -0700] "GET /a?b=c HTTP/1.0" 200 2326 "-" "x"',
             b'garbage line', b'5.6.7.8 - u [31/Dec/2019:23:59:59 +0100] "POST /x#f HTTP/1.1" 404 - "http://h:8/p?q" "y"']
    data = b"".join(l + b"\n" for l in lines * 7)
    st, h = oracle.digest_lines("combined", fields, data, 3, 100)
    assert len(st) == 21
    o = oracle.Oracle("combined", fields)
    for i, l in enumerate(lines * 7):
        s, js = o.parse_raw(l)
        assert st[i] == s
        assert int(h[i]) == (_fnv1a(js.encode()) if s == oracle.OK else 0)
