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


@pytest.mark.parametrize("idx", range(56))
def test_golden_vector(oracle, vectors, idx):
    cases = vectors["cases"]
    if idx >= len(cases):
        pytest.skip("no such case")
    c = cases[idx]
    if c["source"].startswith("hpt/MultiLineHttpdLogParserTest"):
        pytest.skip("sequence case: covered by test_multiline_sequence")
    o = oracle.Oracle(c["logformat"], c["fields"])
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
