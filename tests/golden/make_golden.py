"""Writes tests/golden/reference_vectors.json.

Every case below is TRANSCRIBED DATA (input line, logformat, requested fields,
expected values) from the reference's own JUnit tests; each carries the
reference file:line it comes from (paths relative to /root/reference,
hpt/ = httpdlog/httpdlog-parser/src/test/java/nl/basjes/parse/httpdlog/).
No reference source is copied: only the literal inputs/expectations.

Expectation encoding (mirrors TestRecord's absent / null / value split,
parser-core/src/test/java/nl/basjes/parse/core/test/TestRecord.java:47-114):
  "expect":  {path: value}  value = "str" | null | {"l": n}; the value must be
             among the values delivered for that path
  "absent":  [path, ...]    the path must not be delivered at all
  "bad":     true           the line must raise DissectionFailure
  "remaps":  [[input path, NEW TYPE], ...] the parser's addTypeRemapping calls
Fields the reference test asserts through dissectors this build does not
cover (GeoIP, the Flink example's own ScreenResolutionDissector) are left out
and listed in "skipped".
"""
import json
import os

HERE = os.path.dirname(os.path.abspath(__file__))

CASES = []


# Reference tests written with DissectorTester
# (parser-core/src/test/java/nl/basjes/parse/core/test/DissectorTester.java):
# their .expect(field, (String) null) means "present AND null" (EdgeCasesTest.java:37-46);
# the Map-based record tests (ApacheHttpdLogParserTest, MultiLine, Jetty,
# Flink TestCase) read null for an absent field too.
DISSECTOR_TESTER_SOURCES = ("EdgeCasesTest", "NginxLogFormatTest", "NginxUpstreamTest", "dissectors/Test",
                            "TestTranslators", "AllFieldsTest")


def case(source, logformat, line, fields, expect=None, absent=(), bad=False, skipped=(), note="", remaps=()):
    CASES.append({
        "remaps": [list(r) for r in remaps],
        "source": source,
        "null_present": any(k in source for k in DISSECTOR_TESTER_SOURCES),
        "logformat": logformat,
        "line": line,
        "fields": list(fields),
        "expect": expect or {},
        "absent": list(absent),
        "bad": bad,
        "skipped": list(skipped),
        "note": note,
    })


# --------------------------------------------------------------- Apache whole line
FULLCOMBINED = ("%%%h %a %A %l %u %t \"%r\" %>s %b %p \"%q\" \"%!200,304,302{Referer}i\" %D "
                "\"%200{User-agent}i\" \"%{Cookie}i\" \"%{Set-Cookie}o\" \"%{If-None-Match}i\" \"%{Etag}o\"")
APACHE_TEST_FIELDS = [
    "STRING:request.firstline.uri.query.*", "STRING:request.querystring.aap", "IP:connection.client.ip",
    "NUMBER:connection.client.logname", "STRING:connection.client.user", "TIME.STAMP:request.receive.time",
    "TIME.SECOND:request.receive.time.second", "HTTP.URI:request.firstline.uri", "STRING:request.status.last",
    "BYTESCLF:response.body.bytes", "HTTP.URI:request.referer", "STRING:request.referer.query.mies",
    "STRING:request.referer.query.wim", "HTTP.USERAGENT:request.user-agent", "TIME.DAY:request.receive.time.day",
    "TIME.HOUR:request.receive.time.hour", "TIME.MONTHNAME:request.receive.time.monthname",
    "TIME.EPOCH:request.receive.time.epoch", "TIME.WEEK:request.receive.time.weekofweekyear",
    "TIME.YEAR:request.receive.time.weekyear", "TIME.YEAR:request.receive.time.year",
    "HTTP.COOKIES:request.cookies", "HTTP.SETCOOKIES:response.cookies",
    "MICROSECONDS:response.server.processing.time", "HTTP.HEADER:response.header.etag",
]
APACHE_SKIPPED = ["HTTP.COOKIE:request.cookies.jquery-ui-theme (the (cookies) case below)",
                  "HTTP.SETCOOKIE:response.cookies.apache (the (cookies) case below)",
                  "STRING:response.cookies.apache.domain (the (cookies) case below)",
                  "SCREENWIDTH:request.firstline.uri.query.res.width",
                  "SCREENHEIGHT:request.firstline.uri.query.res.height"]

case("hpt/ApacheHttpdLogParserTest.java:104-163", FULLCOMBINED,
     "%127.0.0.1 127.0.0.1 127.0.0.1 - - [31/Dec/2012:23:49:40 +0100] "
     "\"GET /icons/powered_by_rh.png?aap=noot&res=1024x768 HTTP/1.1\" 200 1213 "
     "80 \"\" \"http://localhost/index.php?mies=wim\" 351 "
     "\"Mozilla/5.0 (X11; Linux i686 on x86_64; rv:11.0) Gecko/20100101 Firefox/11.0\" "
     "\"jquery-ui-theme=Eggplant\" \"Apache=127.0.0.1.1344635380111339; path=/; domain=.basjes.nl\" \"-\" "
     "\"\\\"3780ff-4bd-4c1ce3df91380\\\"\"",
     APACHE_TEST_FIELDS,
     expect={
         "STRING:request.firstline.uri.query.aap": "noot",
         "IP:connection.client.ip": "127.0.0.1",
         "NUMBER:connection.client.logname": None,
         "STRING:connection.client.user": None,
         "TIME.STAMP:request.receive.time": "31/Dec/2012:23:49:40 +0100",
         "TIME.EPOCH:request.receive.time.epoch": {"l": 1356994180000},
         "TIME.WEEK:request.receive.time.weekofweekyear": {"l": 1},
         "TIME.YEAR:request.receive.time.weekyear": {"l": 2013},
         "TIME.YEAR:request.receive.time.year": {"l": 2012},
         "TIME.SECOND:request.receive.time.second": {"l": 40},
         "HTTP.URI:request.firstline.uri": "/icons/powered_by_rh.png?aap=noot&res=1024x768",
         "STRING:request.status.last": "200",
         "BYTESCLF:response.body.bytes": "1213",
         "HTTP.URI:request.referer": "http://localhost/index.php?mies=wim",
         "STRING:request.referer.query.mies": "wim",
         "HTTP.USERAGENT:request.user-agent": "Mozilla/5.0 (X11; Linux i686 on x86_64; rv:11.0) Gecko/20100101 Firefox/11.0",
         "TIME.DAY:request.receive.time.day": {"l": 31},
         "TIME.HOUR:request.receive.time.hour": {"l": 23},
         "TIME.MONTHNAME:request.receive.time.monthname": "December",
         "MICROSECONDS:response.server.processing.time": "351",
         "HTTP.SETCOOKIES:response.cookies": "Apache=127.0.0.1.1344635380111339; path=/; domain=.basjes.nl",
         "HTTP.COOKIES:request.cookies": "jquery-ui-theme=Eggplant",
         "HTTP.HEADER:response.header.etag": "\\\"3780ff-4bd-4c1ce3df91380\\\"",
     },
     absent=["STRING:request.firstline.uri.query.foo", "STRING:request.querystring.aap"],
     skipped=APACHE_SKIPPED)

# the same line's request cookie (RequestCookieListDissector; the Set-Cookie
# dissectors stay off the device and out of the oracle)
case("hpt/ApacheHttpdLogParserTest.java:104-163 (cookies)", FULLCOMBINED,
     "%127.0.0.1 127.0.0.1 127.0.0.1 - - [31/Dec/2012:23:49:40 +0100] "
     "\"GET /icons/powered_by_rh.png?aap=noot&res=1024x768 HTTP/1.1\" 200 1213 "
     "80 \"\" \"http://localhost/index.php?mies=wim\" 351 "
     "\"Mozilla/5.0 (X11; Linux i686 on x86_64; rv:11.0) Gecko/20100101 Firefox/11.0\" "
     "\"jquery-ui-theme=Eggplant\" \"Apache=127.0.0.1.1344635380111339; path=/; domain=.basjes.nl\" \"-\" "
     "\"\\\"3780ff-4bd-4c1ce3df91380\\\"\"",
     ["HTTP.COOKIES:request.cookies", "HTTP.COOKIE:request.cookies.jquery-ui-theme",
      "HTTP.SETCOOKIES:response.cookies", "HTTP.SETCOOKIE:response.cookies.apache",
      "STRING:response.cookies.apache.domain"],
     expect={"HTTP.COOKIES:request.cookies": "jquery-ui-theme=Eggplant",
             "HTTP.COOKIE:request.cookies.jquery-ui-theme": "Eggplant",
             "HTTP.SETCOOKIES:response.cookies": "Apache=127.0.0.1.1344635380111339; path=/; domain=.basjes.nl",
             "HTTP.SETCOOKIE:response.cookies.apache": "Apache=127.0.0.1.1344635380111339; path=/; domain=.basjes.nl",
             "STRING:response.cookies.apache.domain": ".basjes.nl"})

# hpt/CookiesTest.java:110-127,157-218 (cookiesTest): the request cookies of COOKIES_LINE
COOKIES_FMT = ("%h %a %A %l %u %t \"%r\" %>s %b %p \"%q\" \"%{Referer}i\" %D \"%{User-agent}i\" "
               "\"%{Cookie}i\" \"%{Set-Cookie}o\" \"%{If-None-Match}i\" \"%{Etag}o\"")
case("hpt/CookiesTest.java:110-127,157-218", COOKIES_FMT,
     "127.0.0.1 127.0.0.1 127.0.0.1 - - [31/Dec/2012:23:00:44 -0700] \"GET /index.php HTTP/1.1\" "
     "200 - 80 \"\" \"-\" 80991 \"Mozilla/5.0 (X11; Linux i686 on x86_64; rv:11.0) Gecko/20100101 Firefox/11.0\" "
     "\"jquery-ui-theme=Eggplant; Apache=127.0.0.1.1351111543699529\" "
     "\"NBA-0=, NBA-1=1234, NBA-2=1234; expires=Wed, 01-Jan-2020 00:00:10 GMT, "
     "NBA-3=1234; expires=Wed, 01-Jan-2020 00:00:10 GMT; path=/, "
     "NBA-4=1234; expires=Wed, 01-Jan-2020 00:00:10 GMT; path=/; domain=.basj.es\" \"-\" \"-\"",
     ["HTTP.COOKIES:request.cookies", "HTTP.COOKIE:request.cookies.*", "STRING:request.status.last",
      "HTTP.URI:request.firstline.uri"],
     expect={"HTTP.COOKIE:request.cookies.jquery-ui-theme": "Eggplant",
             "HTTP.COOKIE:request.cookies.apache": "127.0.0.1.1351111543699529",
             "STRING:request.status.last": "200", "HTTP.URI:request.firstline.uri": "/index.php"},
     skipped=["HTTP.SETCOOKIES / HTTP.SETCOOKIE fields (the next case)"])

# hpt/CookiesTest.java:71-80,219-232: the Set-Cookie list of COOKIES_LINE
# (ResponseSetCookieListDissector + ResponseSetCookieDissector).  The test
# accepts the expires seconds within 2 (a Double compare); the value is the
# Long 1577836810 (its getString is "1577836810").
case("hpt/CookiesTest.java:71-80,219-232", COOKIES_FMT,
     "127.0.0.1 127.0.0.1 127.0.0.1 - - [31/Dec/2012:23:00:44 -0700] \"GET /index.php HTTP/1.1\" "
     "200 - 80 \"\" \"-\" 80991 \"Mozilla/5.0 (X11; Linux i686 on x86_64; rv:11.0) Gecko/20100101 Firefox/11.0\" "
     "\"jquery-ui-theme=Eggplant; Apache=127.0.0.1.1351111543699529\" "
     "\"NBA-0=, NBA-1=1234, NBA-2=1234; expires=Wed, 01-Jan-2020 00:00:10 GMT, "
     "NBA-3=1234; expires=Wed, 01-Jan-2020 00:00:10 GMT; path=/, "
     "NBA-4=1234; expires=Wed, 01-Jan-2020 00:00:10 GMT; path=/; domain=.basj.es\" \"-\" \"-\"",
     ["HTTP.SETCOOKIES:response.cookies", "HTTP.SETCOOKIE:response.cookies.nba-4", "STRING:response.cookies.nba-4.value",
      "STRING:response.cookies.nba-4.expires", "STRING:response.cookies.nba-4.path",
      "STRING:response.cookies.nba-4.domain"],
     expect={"HTTP.SETCOOKIES:response.cookies":
             "NBA-0=, NBA-1=1234, NBA-2=1234; expires=Wed, 01-Jan-2020 00:00:10 GMT, "
             "NBA-3=1234; expires=Wed, 01-Jan-2020 00:00:10 GMT; path=/, "
             "NBA-4=1234; expires=Wed, 01-Jan-2020 00:00:10 GMT; path=/; domain=.basj.es",
             "HTTP.SETCOOKIE:response.cookies.nba-4": "NBA-4=1234; expires=Wed, 01-Jan-2020 00:00:10 GMT; path=/; domain=.basj.es",
             "STRING:response.cookies.nba-4.value": "1234",
             "STRING:response.cookies.nba-4.expires": {"l": 1577836810},
             "STRING:response.cookies.nba-4.path": "/",
             "STRING:response.cookies.nba-4.domain": ".basj.es"})

# hpt/dissectors/TestCookieDissector.java:43-135 (testResponseSetCookies), as
# the %{Set-Cookie}o token of a one-token LogFormat ("cookies" -> "response.cookies")
_SC_IN = ("NBA-0=, NBA-1=1234, NBA-2=1234; expires=Wed, 01-Jan-2020 00:00:10 GMT, "
          "NBA-3=1234; expires=Wed, 01-Jan-2020 00:00:10 GMT; path=/xx, "
          "NBA-4=1234; expires=Wed, 01-Jan-2020 00:00:10 GMT; path=/xx; domain=.basj.es, "
          "NBA-5=1234; path=/xx; domain=.basj.es, "
          "NBA-6=1234; expires=Wed, 01-Jan-2020 00:00:10 GMT; domain=.basj.es, "
          "NBA-7=1234; expires=Wed, 01-Jan-2020 00:00:10 GMT; domain=.basj.es; comment=bla bla bla")
_SC = {0: ("NBA-0=", "", None, None, None, None), 1: ("NBA-1=1234", "1234", None, None, None, None),
       2: ("NBA-2=1234; expires=Wed, 01-Jan-2020 00:00:10 GMT", "1234", True, None, None, None),
       3: ("NBA-3=1234; expires=Wed, 01-Jan-2020 00:00:10 GMT; path=/xx", "1234", True, "/xx", None, None),
       4: ("NBA-4=1234; expires=Wed, 01-Jan-2020 00:00:10 GMT; path=/xx; domain=.basj.es", "1234", True, "/xx",
           ".basj.es", None),
       5: ("NBA-5=1234; path=/xx; domain=.basj.es", "1234", None, "/xx", ".basj.es", None),
       6: ("NBA-6=1234; expires=Wed, 01-Jan-2020 00:00:10 GMT; domain=.basj.es", "1234", True, None, ".basj.es", None),
       7: ("NBA-7=1234; expires=Wed, 01-Jan-2020 00:00:10 GMT; domain=.basj.es; comment=bla bla bla", "1234", True,
           None, ".basj.es", "bla bla bla")}
_sc_fields, _sc_expect, _sc_absent = ["HTTP.SETCOOKIES:response.cookies"], {"HTTP.SETCOOKIES:response.cookies": _SC_IN}, []
for _k, (_c, _v, _ex, _p, _d, _cm) in _SC.items():
    _b = "response.cookies.nba-%d" % _k
    _sc_fields += ["HTTP.SETCOOKIE:" + _b, "STRING:%s.value" % _b, "STRING:%s.expires" % _b,
                   "TIME.EPOCH:%s.expires" % _b, "STRING:%s.path" % _b, "STRING:%s.domain" % _b,
                   "STRING:%s.comment" % _b]
    _sc_expect["HTTP.SETCOOKIE:" + _b] = _c
    _sc_expect["STRING:%s.value" % _b] = _v
    if _ex:
        _sc_expect["STRING:%s.expires" % _b] = {"l": 1577836810}
        _sc_expect["TIME.EPOCH:%s.expires" % _b] = {"l": 1577836810000}
    else:
        _sc_absent += ["STRING:%s.expires" % _b, "TIME.EPOCH:%s.expires" % _b]
    for _t, _x in (("path", _p), ("domain", _d), ("comment", _cm)):
        if _x is None:
            if _k != 7 or _t == "path":
                _sc_absent.append("STRING:%s.%s" % (_b, _t))
        else:
            _sc_expect["STRING:%s.%s" % (_b, _t)] = _x
case("hpt/dissectors/TestCookieDissector.java:43-135", "%{Set-Cookie}o", _SC_IN, _sc_fields, expect=_sc_expect,
     absent=_sc_absent)

# hpt/dissectors/TestCookieDissector.java:26-40 (testRequestCookies), as the
# %{Cookie}i token of a one-token LogFormat
case("hpt/dissectors/TestCookieDissector.java:26-40", "%{Cookie}i", "NBA-0; NBA-1=; NBA-2=1234; ",
     ["HTTP.COOKIES:request.cookies", "HTTP.COOKIE:request.cookies.nba-0", "HTTP.COOKIE:request.cookies.nba-1",
      "HTTP.COOKIE:request.cookies.nba-2"],
     expect={"HTTP.COOKIES:request.cookies": "NBA-0; NBA-1=; NBA-2=1234; ",
             "HTTP.COOKIE:request.cookies.nba-0": "", "HTTP.COOKIE:request.cookies.nba-1": "",
             "HTTP.COOKIE:request.cookies.nba-2": "1234"})

case("hpt/ApacheHttpdLogParserTest.java:168-200", FULLCOMBINED,
     "%127.0.0.1 127.0.0.1 127.0.0.1 - - [10/Aug/2012:23:55:11 +0200] \"GET /icons/powered_by_rh.png HTTP/1.1\" 200 1213 80"
     " \"\" \"http://localhost/\" 1306 \"Mozilla/5.0 (X11; Linux i686 on x86_64; rv:11.0) Gecko/20100101 Firefox/11.0\""
     " \"jquery-ui-theme=Eggplant; Apache=127.0.0.1.1344635667182858\" \"-\" \"-\" \"\\\"3780ff-4bd-4c1ce3df91380\\\"\"",
     APACHE_TEST_FIELDS,
     expect={
         "IP:connection.client.ip": "127.0.0.1",
         "NUMBER:connection.client.logname": None,
         "STRING:connection.client.user": None,
         "TIME.STAMP:request.receive.time": "10/Aug/2012:23:55:11 +0200",
         "TIME.SECOND:request.receive.time.second": {"l": 11},
         "HTTP.URI:request.firstline.uri": "/icons/powered_by_rh.png",
         "STRING:request.status.last": "200",
         "BYTESCLF:response.body.bytes": "1213",
         "HTTP.URI:request.referer": "http://localhost/",
         "HTTP.USERAGENT:request.user-agent": "Mozilla/5.0 (X11; Linux i686 on x86_64; rv:11.0) Gecko/20100101 Firefox/11.0",
         "TIME.DAY:request.receive.time.day": {"l": 10},
         "TIME.HOUR:request.receive.time.hour": {"l": 23},
         "TIME.MONTHNAME:request.receive.time.monthname": "August",
         "MICROSECONDS:response.server.processing.time": "1306",
         "HTTP.SETCOOKIES:response.cookies": None,
         "HTTP.COOKIES:request.cookies": "jquery-ui-theme=Eggplant; Apache=127.0.0.1.1344635667182858",
         "HTTP.HEADER:response.header.etag": "\\\"3780ff-4bd-4c1ce3df91380\\\"",
     },
     absent=["HTTP.QUERYSTRING:request.firstline.uri.query.foo"])

case("hpt/ApacheHttpdLogParserTest.java:205-239", FULLCOMBINED,
     "%127.0.0.1 127.0.0.1 127.0.0.1 - - [10/Aug/2012:23:55:11 +0200] \"GET /ImagineAURLHereThatIsTooLong\" 414 1213 80"
     " \"\" \"http://localhost/\" 1306 \"Mozilla/5.0 (X11; Linux i686 on x86_64; rv:11.0) Gecko/20100101 Firefox/11.0\""
     " \"jquery-ui-theme=Eggplant; Apache=127.0.0.1.1344635667182858\" \"-\" \"-\" \"\\\"3780ff-4bd-4c1ce3df91380\\\"\"",
     APACHE_TEST_FIELDS,
     expect={
         "IP:connection.client.ip": "127.0.0.1",
         "TIME.STAMP:request.receive.time": "10/Aug/2012:23:55:11 +0200",
         "TIME.SECOND:request.receive.time.second": {"l": 11},
         "HTTP.URI:request.firstline.uri": "/ImagineAURLHereThatIsTooLong",
         "STRING:request.status.last": "414",
         "BYTESCLF:response.body.bytes": "1213",
         "HTTP.URI:request.referer": "http://localhost/",
         "TIME.MONTHNAME:request.receive.time.monthname": "August",
         "MICROSECONDS:response.server.processing.time": "1306",
         "HTTP.SETCOOKIES:response.cookies": None,
         "HTTP.HEADER:response.header.etag": "\\\"3780ff-4bd-4c1ce3df91380\\\"",
     })

QS_FIELDS = ["STRING:request.firstline.uri.query.foo", "STRING:request.firstline.uri.query.bar",
             "HTTP.PATH:request.firstline.uri.path", "HTTP.QUERYSTRING:request.firstline.uri.query",
             "HTTP.REF:request.firstline.uri.ref"]
for line, foo, bar, query, ref, ln in [
    ("GET /index.html HTTP/1.1", "ABSENT", "ABSENT", "", "NULL", "349-354"),
    ("GET /index.html?foo HTTP/1.1", "", "ABSENT", "&foo", "NULL", "357-362"),
    ("GET /index.html&foo HTTP/1.1", "", "ABSENT", "&foo", "NULL", "365-370"),
    ("GET /index.html?foo=foofoo# HTTP/1.1", "foofoo", "ABSENT", "&foo=foofoo", "", "373-378"),
    ("GET /index.html&foo=foofoo HTTP/1.1", "foofoo", "ABSENT", "&foo=foofoo", "NULL", "381-386"),
    ("GET /index.html?bar&foo=foofoo# HTTP/1.1", "foofoo", "", "&bar&foo=foofoo", "", "389-394"),
    ("GET /index.html?bar&foo=foofoo#bookmark HTTP/1.1", "foofoo", "", "&bar&foo=foofoo", "bookmark", "397-402"),
    ("GET /index.html?bar=barbar&foo=foofoo#bookmark HTTP/1.1", "foofoo", "barbar", "&bar=barbar&foo=foofoo", "bookmark", "405-410"),
    ("GET /index.html&bar=barbar&foo=foofoo#bla HTTP/1.1", "foofoo", "barbar", "&bar=barbar&foo=foofoo", "bla", "413-418"),
    ("GET /index.html&bar=barbar?foo=foofoo HTTP/1.1", "foofoo", "barbar", "&bar=barbar&foo=foofoo", "NULL", "421-426"),
]:
    exp = {"HTTP.PATH:request.firstline.uri.path": "/index.html", "HTTP.QUERYSTRING:request.firstline.uri.query": query}
    absent = []
    for k, v in (("STRING:request.firstline.uri.query.foo", foo), ("STRING:request.firstline.uri.query.bar", bar),
                 ("HTTP.REF:request.firstline.uri.ref", ref)):
        if v == "ABSENT":
            absent.append(k)
        elif v == "NULL":
            exp[k] = None
        else:
            exp[k] = v
    case("hpt/ApacheHttpdLogParserTest.java:" + ln, "%r", line, QS_FIELDS, expect=exp, absent=absent,
         note="Map-based test record: a null assert may mean absent or null; both accepted as reference encodes")

case("hpt/EdgeCasesTest.java:26-57",
     "%a %{Host}i %u %t \"%r\" %>s %O \"%{Referer}i\" \"%{User-Agent}i\" %{Content-length}i %P %A",
     "1.2.3.4 - - [03/Apr/2017:03:27:28 -0600] \"\\x16\\x03\\x01\" 404 419 \"-\" \"-\" - 115052 5.6.7.8",
     ["IP:connection.client.ip", "IP:connection.server.ip", "TIME.EPOCH:request.receive.time.last.epoch",
      "STRING:connection.client.user", "TIME.STAMP:request.receive.time.last", "TIME.DATE:request.receive.time.last.date",
      "TIME.TIME:request.receive.time.last.time", "NUMBER:connection.server.child.processid", "BYTES:response.bytes",
      "STRING:request.status.last", "HTTP.USERAGENT:request.user-agent", "HTTP.HEADER:request.header.host",
      "HTTP.HEADER:request.header.content-length", "HTTP.URI:request.referer", "HTTP.FIRSTLINE:request.firstline",
      "HTTP.METHOD:request.firstline.method", "HTTP.URI:request.firstline.uri", "HTTP.PROTOCOL:request.firstline.protocol"],
     expect={
         "IP:connection.client.ip": "1.2.3.4",
         "IP:connection.server.ip": "5.6.7.8",
         "TIME.EPOCH:request.receive.time.last.epoch": {"l": 1491211648000},
         "STRING:connection.client.user": None,
         "TIME.STAMP:request.receive.time.last": "03/Apr/2017:03:27:28 -0600",
         "TIME.DATE:request.receive.time.last.date": "2017-04-03",
         "TIME.TIME:request.receive.time.last.time": "03:27:28",
         "NUMBER:connection.server.child.processid": "115052",
         "BYTES:response.bytes": "419",
         "STRING:request.status.last": "404",
         "HTTP.USERAGENT:request.user-agent": None,
         "HTTP.HEADER:request.header.host": None,
         "HTTP.HEADER:request.header.content-length": None,
         "HTTP.URI:request.referer": None,
         "HTTP.FIRSTLINE:request.firstline": "\\x16\\x03\\x01",
     },
     absent=["HTTP.METHOD:request.firstline.method", "HTTP.URI:request.firstline.uri",
             "HTTP.PROTOCOL:request.firstline.protocol"])

# Multi-format sticky switching (hpt/MultiLineHttpdLogParserTest.java:64-124)
ML_FMT = "%h %t \"%r\" %>s %b \"%{Referer}i\"\n\n%h %t \"%r\" %>s \"%{User-Agent}i\"\n\n"
ML_FIELDS = ["IP:connection.client.host", "TIME.STAMP:request.receive.time", "TIME.SECOND:request.receive.time.second",
             "STRING:request.status.last", "BYTESCLF:response.body.bytes", "HTTP.URI:request.firstline.uri",
             "HTTP.URI:request.referer", "HTTP.USERAGENT:request.user-agent"]
ML_L1 = ("127.0.0.1 [31/Dec/2012:23:49:41 +0100] \"GET /foo HTTP/1.1\" 200 1213 \"http://localhost/index.php?mies=wim\"")
ML_L2 = ("127.0.0.2 [31/Dec/2012:23:49:42 +0100] \"GET /foo HTTP/1.1\" 404 "
         "\"Mozilla/5.0 (X11; Linux i686 on x86_64; rv:11.0) Gecko/20100101 Firefox/11.0\"")
ML_E1 = {"IP:connection.client.host": "127.0.0.1", "TIME.STAMP:request.receive.time": "31/Dec/2012:23:49:41 +0100",
         "HTTP.URI:request.firstline.uri": "/foo", "STRING:request.status.last": "200",
         "BYTESCLF:response.body.bytes": "1213", "HTTP.URI:request.referer": "http://localhost/index.php?mies=wim"}
ML_E2 = {"IP:connection.client.host": "127.0.0.2", "TIME.STAMP:request.receive.time": "31/Dec/2012:23:49:42 +0100",
         "HTTP.URI:request.firstline.uri": "/foo", "STRING:request.status.last": "404",
         "HTTP.USERAGENT:request.user-agent": "Mozilla/5.0 (X11; Linux i686 on x86_64; rv:11.0) Gecko/20100101 Firefox/11.0"}
for i, which in enumerate([1, 1, 2, 2, 1, 1, 2, 2, 1, 1, 2, 2]):
    case("hpt/MultiLineHttpdLogParserTest.java:64-124 (sequence step %d)" % i, ML_FMT, ML_L1 if which == 1 else ML_L2,
         ML_FIELDS, expect=ML_E1 if which == 1 else ML_E2,
         absent=["HTTP.USERAGENT:request.user-agent"] if which == 1 else ["BYTESCLF:response.body.bytes", "HTTP.URI:request.referer"],
         note="sequence: one parser for all 12 steps (sticky active format)")

# Jetty fix (hpt/JettyLogFormatParserTest.java:62-104): "ENABLE JETTY FIX" adds patched formats
JETTY_FMT = "ENABLE JETTY FIX\n%h %l %u %t \"%r\" %>s %b \"%{Referer}i\" \"%{User-Agent}i\" %D"
JETTY_FIELDS = ["IP:connection.client.host", "NUMBER:connection.client.logname", "STRING:connection.client.user",
                "TIME.STAMP:request.receive.time", "TIME.DAY:request.receive.time.day", "HTTP.FIRSTLINE:request.firstline",
                "STRING:request.status.last", "BYTES:response.body.bytes", "HTTP.URI:request.referer",
                "HTTP.USERAGENT:request.user-agent", "MICROSECONDS:response.server.processing.time"]
JETTY_LINES = [  # (line, user, user-agent) -- the test's four lines, verbatim
    ("0.0.0.0 - x [24/Jul/2016:07:08:31 +0000] \"GET http://[:1]/foo HTTP/1.1\" 400 0 \"http://other.site\" \"-\"  8", "x", None),
    ("0.0.0.0 -  -  [24/Jul/2016:07:08:31 +0000] \"GET http://[:1]/foo HTTP/1.1\" 400 0 \"http://other.site\" \"-\"  8", None, None),
    ("0.0.0.0 - x [24/Jul/2016:07:08:31 +0000] \"GET http://[:1]/foo HTTP/1.1\" 400 0 \"http://other.site\" \"Mozilla/5.0 (dummy)\" 8",
     "x", "Mozilla/5.0 (dummy)"),
    ("0.0.0.0 -  -  [24/Jul/2016:07:08:31 +0000] \"GET http://[:1]/foo HTTP/1.1\" 400 0 \"http://other.site\" \"Mozilla/5.0 (dummy)\" 8",
     None, "Mozilla/5.0 (dummy)")]
for line, user_v, ua_v in JETTY_LINES:
    case("hpt/JettyLogFormatParserTest.java:62-104", JETTY_FMT, line, JETTY_FIELDS,
         expect={"IP:connection.client.host": "0.0.0.0", "NUMBER:connection.client.logname": None,
                 "STRING:connection.client.user": user_v, "TIME.STAMP:request.receive.time": "24/Jul/2016:07:08:31 +0000",
                 "TIME.DAY:request.receive.time.day": {"l": 24}, "HTTP.FIRSTLINE:request.firstline": "GET http://[:1]/foo HTTP/1.1",
                 "STRING:request.status.last": "400", "BYTES:response.body.bytes": "0",
                 "HTTP.URI:request.referer": "http://other.site", "HTTP.USERAGENT:request.user-agent": ua_v,
                 "MICROSECONDS:response.server.processing.time": "8"},
         note="each line parsed by a fresh parser (the test's assertions hold for any routing order)")

# ------------------------------------------------------- component-level (via one-token formats)
# HttpUriDissector tests (hpt/dissectors/TestHttpUriDissector.java) through "%{referer}i": the line is the URI.
URI_PFX = "request.referer."
URI_F = ["HTTP.PROTOCOL:protocol", "HTTP.USERINFO:userinfo", "HTTP.HOST:host", "HTTP.PORT:port", "HTTP.PATH:path",
         "HTTP.QUERYSTRING:query", "HTTP.REF:ref"]


def uri_case(ln, uri, exp, absent=(), extra_fields=()):
    def pfx(f):
        t, n = f.split(":", 1)
        return t + ":" + URI_PFX + n
    fields = [pfx(f) for f in URI_F] + [pfx(f) for f in extra_fields]
    case("hpt/dissectors/TestHttpUriDissector.java:" + ln, "%{referer}i", uri, fields,
         expect={pfx(k): v for k, v in exp.items()}, absent=[pfx(a) for a in absent])


uri_case("25-40", "http://www.example.com/some/thing/else/index.html?foofoo=bar%20bar",
         {"HTTP.PROTOCOL:protocol": "http", "HTTP.USERINFO:userinfo": None, "HTTP.HOST:host": "www.example.com",
          "HTTP.PATH:path": "/some/thing/else/index.html", "HTTP.QUERYSTRING:query": "&foofoo=bar%20bar",
          "HTTP.REF:ref": None}, absent=["HTTP.PORT:port"])
uri_case("42-57", "http://www.example.com/some/thing/else/index.html&aap=noot?foofoo=barbar&",
         {"HTTP.PROTOCOL:protocol": "http", "HTTP.USERINFO:userinfo": None, "HTTP.HOST:host": "www.example.com",
          "HTTP.PATH:path": "/some/thing/else/index.html", "HTTP.QUERYSTRING:query": "&aap=noot&foofoo=barbar&",
          "HTTP.REF:ref": None}, absent=["HTTP.PORT:port"])
uri_case("59-74", "http://www.example.com:8080/some/thing/else/index.html&aap=noot?foofoo=barbar&#blabla",
         {"HTTP.PROTOCOL:protocol": "http", "HTTP.USERINFO:userinfo": None, "HTTP.HOST:host": "www.example.com",
          "HTTP.PORT:port": {"l": 8080}, "HTTP.PATH:path": "/some/thing/else/index.html",
          "HTTP.QUERYSTRING:query": "&aap=noot&foofoo=barbar&", "HTTP.REF:ref": "blabla"})
uri_case("76-91", "/some/thing/else/index.html?foofoo=barbar#blabla",
         {"HTTP.PATH:path": "/some/thing/else/index.html", "HTTP.QUERYSTRING:query": "&foofoo=barbar", "HTTP.REF:ref": "blabla"},
         absent=["HTTP.PROTOCOL:protocol", "HTTP.USERINFO:userinfo", "HTTP.HOST:host", "HTTP.PORT:port"])
uri_case("93-108", "/some/thing/else/index.html&aap=noot?foofoo=bar%20bar&#bla%20bla",
         {"HTTP.PATH:path": "/some/thing/else/index.html", "HTTP.QUERYSTRING:query": "&aap=noot&foofoo=bar%20bar&",
          "HTTP.REF:ref": "bla bla"},
         absent=["HTTP.PROTOCOL:protocol", "HTTP.USERINFO:userinfo", "HTTP.HOST:host", "HTTP.PORT:port"])
uri_case("110-125", "android-app://com.google.android.googlequicksearchbox",
         {"HTTP.PROTOCOL:protocol": "android-app", "HTTP.USERINFO:userinfo": None,
          "HTTP.HOST:host": "com.google.android.googlequicksearchbox", "HTTP.PATH:path": "",
          "HTTP.QUERYSTRING:query": "", "HTTP.REF:ref": None}, absent=["HTTP.PORT:port"])
uri_case("127-142", "android-app://com.google.android.googlequicksearchbox/https/www.google.com",
         {"HTTP.PROTOCOL:protocol": "android-app", "HTTP.USERINFO:userinfo": None,
          "HTTP.HOST:host": "com.google.android.googlequicksearchbox", "HTTP.PATH:path": "/https/www.google.com",
          "HTTP.QUERYSTRING:query": "", "HTTP.REF:ref": None}, absent=["HTTP.PORT:port"])
uri_case("144-160", "/some/thing/else/[index.html&aap=noot?foofoo=bar%20bar #bla%20bla ",
         {"HTTP.PATH:path": "/some/thing/else/[index.html", "HTTP.QUERYSTRING:query": "&aap=noot&foofoo=bar%20bar%20",
          "HTTP.REF:ref": "bla bla "},
         absent=["HTTP.PROTOCOL:protocol", "HTTP.USERINFO:userinfo", "HTTP.HOST:host", "HTTP.PORT:port"])
uri_case("162-179", "/index.html&promo=Give-50%-discount&promo=And-do-%Another-Wrong&last=also bad %#bla%20bla ",
         {"HTTP.PATH:path": "/index.html",
          "HTTP.QUERYSTRING:query": "&promo=Give-50%25-discount&promo=And-do-%25Another-Wrong&last=also%20bad%20%25",
          "HTTP.REF:ref": "bla bla "},
         absent=["HTTP.PROTOCOL:protocol", "HTTP.USERINFO:userinfo", "HTTP.HOST:host", "HTTP.PORT:port"])
uri_case("181-198", "/index.html?Linkid=%%%3dv(%40Foo)%3d%%%&emcid=B%ar",
         {"HTTP.PATH:path": "/index.html", "HTTP.QUERYSTRING:query": "&Linkid=%25%25%3dv(%40Foo)%3d%25%25%25&emcid=B%25ar",
          "STRING:query.linkid": "%%=v(@Foo)=%%%", "HTTP.REF:ref": None},
         absent=["HTTP.PROTOCOL:protocol", "HTTP.USERINFO:userinfo", "HTTP.HOST:host", "HTTP.PORT:port"],
         extra_fields=["STRING:query.linkid"])
for u in ["https://www.basjes.nl/#foo#bar#bazz#bla#bla#",
          "https://www.basjes.nl/path/?s2a=&Referrer=ADV1234#product_title&f=API&subid=?s2a=#product_title&name=12341234",
          "https://www.basjes.nl/path/?Referrer=ADV1234#&f=API&subid=#&name=12341234",
          "https://www.basjes.nl/path?sort&#x3D;price&filter&#x3D;new&sortOrder&#x3D;asc",
          "https://www.basjes.nl/login.html?redirectUrl=https%3A%2F%2Fwww.basjes.nl%2Faccount%2Findex.html"
          "&_requestid=1234#x3D;12341234&Referrer&#x3D;ENTblablabla"]:
    uri_case("200-213", u, {"HTTP.HOST:host": "www.basjes.nl"})

# QueryStringFieldDissector (hpt/dissectors/TestQueryStringDissector.java:26-42)
case("hpt/dissectors/TestQueryStringDissector.java:26-42", "%{referer}i",
     "/some/thing/else/index.html&aap=1&noot=&mies&",
     ["HTTP.PATH:request.referer.path", "HTTP.QUERYSTRING:request.referer.query",
      "STRING:request.referer.query.aap", "STRING:request.referer.query.noot", "STRING:request.referer.query.mies",
      "STRING:request.referer.query.wim"],
     expect={"HTTP.PATH:request.referer.path": "/some/thing/else/index.html",
             "HTTP.QUERYSTRING:request.referer.query": "&aap=1&noot=&mies&",
             "STRING:request.referer.query.aap": "1", "STRING:request.referer.query.noot": "",
             "STRING:request.referer.query.mies": ""},
     absent=["STRING:request.referer.query.wim"])

# HttpFirstLineDissector (hpt/dissectors/TestHttpFirstLineDissector.java) through "%r"
FL_F = ["HTTP.METHOD:request.firstline.method", "HTTP.URI:request.firstline.uri",
        "HTTP.PROTOCOL:request.firstline.protocol", "HTTP.PROTOCOL.VERSION:request.firstline.protocol.version"]
case("hpt/dissectors/TestHttpFirstLineDissector.java:25-36", "%r", "GET /index.html HTTP/1.1", FL_F,
     expect={"HTTP.METHOD:request.firstline.method": "GET", "HTTP.URI:request.firstline.uri": "/index.html",
             "HTTP.PROTOCOL:request.firstline.protocol": "HTTP", "HTTP.PROTOCOL.VERSION:request.firstline.protocol.version": "1.1"})
case("hpt/dissectors/TestHttpFirstLineDissector.java:38-48", "%r", "GET /index.html HTT", FL_F,
     expect={"HTTP.METHOD:request.firstline.method": "GET", "HTTP.URI:request.firstline.uri": "/index.html HTT"},
     absent=["HTTP.PROTOCOL:request.firstline.protocol", "HTTP.PROTOCOL.VERSION:request.firstline.protocol.version"])
case("hpt/dissectors/TestHttpFirstLineDissector.java:50-58", "%r", "\\x16\\x03\\x01", FL_F,
     absent=["HTTP.METHOD:request.firstline.method", "HTTP.URI:request.firstline.uri"])
case("hpt/dissectors/TestHttpFirstLineDissector.java:60-71", "%r", "VERSION-CONTROL /index.html HTTP/1.1", FL_F,
     expect={"HTTP.METHOD:request.firstline.method": "VERSION-CONTROL", "HTTP.URI:request.firstline.uri": "/index.html",
             "HTTP.PROTOCOL:request.firstline.protocol": "HTTP", "HTTP.PROTOCOL.VERSION:request.firstline.protocol.version": "1.1"})

# TimeStampDissector (hpt/dissectors/TestTimeStampDissector.java) through "%t" (line = "[ts]")
TS = "request.receive.time."
TS_F = ["TIME.EPOCH:epoch", "TIME.YEAR:year", "TIME.MONTH:month", "TIME.MONTHNAME:monthname", "TIME.DAY:day",
        "TIME.HOUR:hour", "TIME.MINUTE:minute", "TIME.SECOND:second", "TIME.DATE:date", "TIME.TIME:time",
        "TIME.YEAR:year_utc", "TIME.MONTH:month_utc", "TIME.MONTHNAME:monthname_utc", "TIME.DAY:day_utc",
        "TIME.HOUR:hour_utc", "TIME.MINUTE:minute_utc", "TIME.SECOND:second_utc", "TIME.DATE:date_utc",
        "TIME.TIME:time_utc"]


def tsf(f):
    t, n = f.split(":", 1)
    return t + ":" + TS + n


case("hpt/dissectors/TestTimeStampDissector.java:46-86", "%t", "[31/Dec/2012:23:00:44 -0700]", [tsf(f) for f in TS_F],
     expect={tsf(k): v for k, v in {
         "TIME.EPOCH:epoch": {"l": 1357020044000}, "TIME.YEAR:year": {"l": 2012}, "TIME.MONTH:month": {"l": 12},
         "TIME.MONTHNAME:monthname": "December", "TIME.DAY:day": {"l": 31}, "TIME.HOUR:hour": {"l": 23},
         "TIME.MINUTE:minute": {"l": 0}, "TIME.SECOND:second": {"l": 44}, "TIME.DATE:date": "2012-12-31",
         "TIME.TIME:time": "23:00:44", "TIME.YEAR:year_utc": {"l": 2013}, "TIME.MONTH:month_utc": {"l": 1},
         "TIME.MONTHNAME:monthname_utc": "January", "TIME.DAY:day_utc": {"l": 1}, "TIME.HOUR:hour_utc": {"l": 6},
         "TIME.MINUTE:minute_utc": {"l": 0}, "TIME.SECOND:second_utc": {"l": 44}, "TIME.DATE:date_utc": "2013-01-01",
         "TIME.TIME:time_utc": "06:00:44"}.items()})
for m in ["sep", "Sep", "sEp", "SEp", "seP", "SeP", "sEP", "SEP"]:
    case("hpt/dissectors/TestTimeStampDissector.java:150-169", "%t", "[30/%s/2016:00:00:06 +0000]" % m,
         [tsf("TIME.YEAR:year_utc"), tsf("TIME.MONTH:month_utc"), tsf("TIME.DAY:day_utc")],
         expect={tsf("TIME.YEAR:year_utc"): {"l": 2016}, tsf("TIME.MONTH:month_utc"): {"l": 9},
                 tsf("TIME.DAY:day_utc"): {"l": 30}})

# StrfTimeStampDissector (hpt/dissectors/TestTimeStampDissector.java) through "%{...}t" tokens
STRF_EXPECT = {
    "TIME.EPOCH:epoch": {"l": 1357020044000}, "TIME.YEAR:year": {"l": 2012}, "TIME.MONTH:month": {"l": 12},
    "TIME.MONTHNAME:monthname": "December", "TIME.DAY:day": {"l": 31}, "TIME.HOUR:hour": {"l": 23},
    "TIME.MINUTE:minute": {"l": 0}, "TIME.SECOND:second": {"l": 44}, "TIME.DATE:date": "2012-12-31",
    "TIME.TIME:time": "23:00:44", "TIME.YEAR:year_utc": {"l": 2013}, "TIME.MONTH:month_utc": {"l": 1},
    "TIME.MONTHNAME:monthname_utc": "January", "TIME.DAY:day_utc": {"l": 1}, "TIME.HOUR:hour_utc": {"l": 6},
    "TIME.MINUTE:minute_utc": {"l": 0}, "TIME.SECOND:second_utc": {"l": 44}, "TIME.DATE:date_utc": "2013-01-01",
    "TIME.TIME:time_utc": "06:00:44"}
case("hpt/dissectors/TestTimeStampDissector.java:185-226", "%{%Y-%m-%dT%H:%M:%S%z}t", "2012-12-31T23:00:44-0700",
     [tsf(f) for f in TS_F], expect={tsf(k): v for k, v in STRF_EXPECT.items()})
case("hpt/dissectors/TestTimeStampDissector.java:228-235", "%{begin:%Y-%m-%dT%H:%M:%S%z}t", "2012-12-31T23:00:44-0700",
     ["TIME.EPOCH:request.receive.time.begin.epoch"],
     expect={"TIME.EPOCH:request.receive.time.begin.epoch": {"l": 1357020044000}})
case("hpt/dissectors/TestTimeStampDissector.java:237-244", "%{end:%Y-%m-%dT%H:%M:%S%z}t", "2012-12-31T23:00:44-0700",
     ["TIME.EPOCH:request.receive.time.end.epoch"],
     expect={"TIME.EPOCH:request.receive.time.end.epoch": {"l": 1357020044000}})
case("hpt/dissectors/TestTimeStampDissector.java:351-372", "%{%d/%b/%Y %T.msec_frac %z}t", "01/Jan/2017 21:52:58.483 +0100",
     [tsf("TIME.EPOCH:epoch")], expect={tsf("TIME.EPOCH:epoch"): {"l": 1483303978483}})
case("hpt/dissectors/TestTimeStampDissector.java:374-384", "%{%d/%b/%Y:%H:%M:%S %z}t", "28/feb/2017:03:39:40 +0800",
     [tsf("TIME.EPOCH:epoch")], expect={tsf("TIME.EPOCH:epoch"): {"l": 1488224380000}})
case("hpt/dissectors/TestTimeStampDissector.java:524-530", "%{%F %H:%M:%S}t", "2017-12-25 00:00:00",
     [tsf("TIME.EPOCH:epoch")], expect={tsf("TIME.EPOCH:epoch"): {"l": 1514160000000}})
STRF_LINE_FMT = "%a %l %u {} \"%r\" %>s %b \"%{{Referer}}i\" \"%{{User-Agent}}i\" \"%{{Cookie}}i\" t=%D"
case("hpt/dissectors/TestTimeStampDissector.java:532-537", STRF_LINE_FMT.format("%{%F %H:%M:%S}t"),
     "192.168.85.3 - - 2017-12-25 00:00:00 \"GET /up.html HTTP/1.0\" 203 8 \"-\" \"HTTP-Monitor/1.1\" \"-\" t=4920",
     [tsf("TIME.EPOCH:epoch")], expect={tsf("TIME.EPOCH:epoch"): {"l": 1514160000000}})
FRAC_F = ["TIME.EPOCH:epoch", "TIME.SECOND:second", "TIME.MILLISECOND:millisecond", "TIME.MICROSECOND:microsecond",
          "TIME.NANOSECOND:nanosecond", "TIME.MILLISECOND:millisecond_utc", "TIME.MICROSECOND:microsecond_utc",
          "TIME.NANOSECOND:nanosecond_utc"]
for src, frac, digits, ms, us, ns, epoch in [
        ("hpt/dissectors/TestTimeStampDissector.java:540-555", "msec_frac", "123", 123, 123000, 123000000, 1514160042123),
        ("hpt/dissectors/TestTimeStampDissector.java:557-572", "%msec_frac", "123", 123, 123000, 123000000, 1514160042123),
        ("hpt/dissectors/TestTimeStampDissector.java:574-589", "usec_frac", "123456", 123, 123456, 123456000, 1514160042123),
        ("hpt/dissectors/TestTimeStampDissector.java:591-606", "%usec_frac", "123456", 123, 123456, 123456000, 1514160042123)]:
    vals = [{"l": epoch}, {"l": 42}, {"l": ms}, {"l": us}, {"l": ns}, {"l": ms}, {"l": us}, {"l": ns}]
    case(src, STRF_LINE_FMT.format("%{%F %H:%M:%S." + frac + "}t"),
         "192.168.85.3 - - 2017-12-25 00:00:42." + digits + " \"GET /up.html HTTP/1.0\" 203 8 \"-\" \"HTTP-Monitor/1.1\" \"-\" t=4920",
         [tsf(f) for f in FRAC_F], expect={tsf(f): v for f, v in zip(FRAC_F, vals)})
# testSpecialTimeFormatMultiFields1/2, testSpecialTimeLeadingSpaces1/2a: every convertible conversion at once
MULTI_F = ["TIME.EPOCH:epoch", "TIME.DATE:date", "TIME.TIME:time", "TIME.YEAR:year", "TIME.MONTH:month",
           "TIME.MONTHNAME:monthname", "TIME.YEAR:weekyear", "TIME.WEEK:weekofweekyear", "TIME.DAY:day", "TIME.HOUR:hour",
           "TIME.MINUTE:minute", "TIME.SECOND:second", "TIME.MILLISECOND:millisecond", "TIME.DATE:date_utc",
           "TIME.TIME:time_utc", "TIME.YEAR:year_utc", "TIME.MONTH:month_utc", "TIME.MONTHNAME:monthname_utc",
           "TIME.YEAR:weekyear_utc", "TIME.WEEK:weekofweekyear_utc", "TIME.DAY:day_utc", "TIME.HOUR:hour_utc",
           "TIME.MINUTE:minute_utc", "TIME.SECOND:second_utc", "TIME.MILLISECOND:millisecond_utc"]
MULTI_FMT = "%D %F %R %T %r %a %A %b %B %d %G %h %H %I %j %k %l %m %M %p %s %S %u %Y %z"
for src, fmt, line, vals in [
        ("hpt/dissectors/TestTimeStampDissector.java:246-287", "%{" + MULTI_FMT + "}t",
         "12/21/16 2016-12-21 20:50 20:50:25 08:50:25 PM Wed Wednesday Dec December 21 2016 Dec 20 08 356 20  8 12 50 PM "
         "1482349825 25 3 2016 +0100",
         [{"l": 1482349825000}, "2016-12-21", "20:50:25", {"l": 2016}, {"l": 12}, "December", {"l": 2016}, {"l": 51},
          {"l": 21}, {"l": 20}, {"l": 50}, {"l": 25}, {"l": 0}, "2016-12-21", "19:50:25", {"l": 2016}, {"l": 12},
          "December", {"l": 2016}, {"l": 51}, {"l": 21}, {"l": 19}, {"l": 50}, {"l": 25}, {"l": 0}]),
        ("hpt/dissectors/TestTimeStampDissector.java:289-330",
         "%h %l %u %t \"%r\" %>s %O \"%{" + MULTI_FMT + "}t\" \"%{User-Agent}i\"",
         "127.0.0.1 - - [22/Dec/2016:00:09:54 +0100] \"GET / HTTP/1.1\" 200 3525 \"12/22/16 2016-12-22 00:09 00:09:54 "
         "12:09:54 AM Thu Thursday Dec December 22 2016 Dec 00 12 357  0 12 12 09 AM 1482361794 54 4 2016 +0100\" "
         "\"Mozilla/5.0 (X11; Linux x86_64) AppleWebKit/537.36 (KHTML, like Gecko) Chrome/54.0.2840.71 Safari/537.36\"",
         [{"l": 1482361794000}, "2016-12-22", "00:09:54", {"l": 2016}, {"l": 12}, "December", {"l": 2016}, {"l": 51},
          {"l": 22}, {"l": 0}, {"l": 9}, {"l": 54}, {"l": 0}, "2016-12-21", "23:09:54", {"l": 2016}, {"l": 12},
          "December", {"l": 2016}, {"l": 51}, {"l": 21}, {"l": 23}, {"l": 9}, {"l": 54}, {"l": 0}])]:
    case(src, fmt, line, [tsf(f) for f in MULTI_F] + [tsf("TIME.ZONE:timezone")],
         expect={tsf(f): v for f, v in zip(MULTI_F, vals)}, absent=[tsf("TIME.ZONE:timezone")])
case("hpt/dissectors/TestTimeStampDissector.java:332-341", "%{" + MULTI_FMT + "}t",
     "12/21/16 2016-12-21 20:50 20:50:25 08:50:25 PM Wed Wednesday Dec December 21 2016 Dec 20 08 356 20  8 12 50 PM "
     "1482349825 25 3 2016 +0100", [tsf("TIME.EPOCH:epoch")], expect={tsf("TIME.EPOCH:epoch"): {"l": 1482349825000}})
case("hpt/dissectors/TestTimeStampDissector.java:343-352",
     "%h %l %u %t \"%r\" %>s %O \"%{%D %F %R %T %r %a %A %b %B %d %G %h %H %I %j %k %l %m %M %p %S %u %Y %z}t\" "
     "\"%{User-Agent}i\"",
     "127.0.0.1 - - [01/Jan/2017:13:01:21 +0100] \"GET / HTTP/1.1\" 200 3525 \"01/01/17 2017-01-01 13:01 13:01:21 01:01:21 PM "
     "Sun Sunday Jan January 01 2017 Jan 13 01 001 13  1 01 01 PM 21 7 2017 +0100\" \"Mozilla/5.0 (X11; Linux x86_64) "
     "AppleWebKit/537.36 (KHTML, like Gecko) Chrome/54.0.2840.71 Safari/537.36\"",
     [tsf("TIME.EPOCH:epoch")], expect={tsf("TIME.EPOCH:epoch"): {"l": 1483272081000}})
# testAllStrfFieldsLowValues / HighValues (:392-510) pin what each conversion PRINTS for one ZonedDateTime
# (CET, +01:00 on both dates); parsing the printed fields back, joined by spaces, must give that instant.
ALL_FMT = "%a %A %b %h %B %d %D %e %F %G %g %H %I %j %k %l %m %M %p %P %r %R %s %S %T %u %V %W %y %Y %z %T.msec_frac"
for src, text, epoch in [
        ("hpt/dissectors/TestTimeStampDissector.java:392-443 (printed fields parsed back)",
         "Tue Tuesday Jan Jan January 02 01/02/01  2 2001-01-02 2001 01 03 03 002  3  3 01 04 AM am 03:04:05 AM 03:04 "
         "978401045 05 03:04:05 2 1 01 01 2001 +0100 03:04:05.678", 978401045678),
        ("hpt/dissectors/TestTimeStampDissector.java:446-497 (printed fields parsed back)",
         "Sun Sunday Nov Nov November 12 11/12/17 12 2017-11-12 2017 17 23 11 316 23 11 11 14 PM pm 11:14:15 PM 23:14 "
         "1510524855 15 23:14:15 7 45 45 17 2017 +0100 23:14:15.678", 1510524855678)]:
    case(src, "%{" + ALL_FMT + "}t", text, [tsf("TIME.EPOCH:epoch")], expect={tsf("TIME.EPOCH:epoch"): {"l": epoch}},
         note="derived: the concatenation of the checkStrfField outputs of the same date-time")

# examples/apache-flink/.../TestCase.java:37-60,86-94 (IPv6 %h, long query string, the query parameters g and r
# remapped to HTTP.URI and dissected again, s to the example's SCREENRESOLUTION); GeoIP / screen size skipped.
FLINK_LINE = open(os.path.join(HERE, "flink_testcase_line.txt"), encoding="utf-8").read().rstrip("\n") \
    if os.path.exists(os.path.join(HERE, "flink_testcase_line.txt")) else None
if FLINK_LINE:
    case("examples/apache-flink/src/test/java/nl/basjes/parse/httpdlog/flink/TestCase.java:37-60,86-94",
         "%h %l %u %t \"%r\" %>s %b \"%{Referer}i\" \"%{User-Agent}i\" \"%{Cookie}i\"", FLINK_LINE,
         ["IP:connection.client.host", "TIME.STAMP:request.receive.time", "TIME.EPOCH:request.receive.time.epoch",
          "HTTP.USERAGENT:request.user-agent", "STRING:request.firstline.uri.query.g", "STRING:request.firstline.uri.query.s",
          "HTTP.COOKIE:request.cookies.bui", "STRING:request.firstline.uri.query.g.query.promo",
          "STRING:request.firstline.uri.query.r.query.blabla"],
         expect={"IP:connection.client.host": "2001:980:91c0:1:8d31:a232:25e5:85d",
                 "TIME.STAMP:request.receive.time": "05/Sep/2010:11:27:50 +0200",
                 "TIME.EPOCH:request.receive.time.epoch": {"l": 1283678870000},
                 "STRING:request.firstline.uri.query.s": "1280x800",
                 "HTTP.USERAGENT:request.user-agent": "Mozilla/5.0 (Macintosh; U; Intel Mac OS X 10_6_4; nl-nl) "
                                                      "AppleWebKit/533.17.8 (KHTML, like Gecko) Version/5.0.1 Safari/533.17.8",
                 "HTTP.COOKIE:request.cookies.bui": "SomeThing",
                 # getExpectedReferrer / getExpectedGoogleQuery (:88, :92)
                 "STRING:request.firstline.uri.query.g.query.promo":
                     "koken-pannen_303_hs-koken-pannen-afj-120601_B3_product_1_9200000002876066",
                 "STRING:request.firstline.uri.query.r.query.blabla": "blablawashere"},
         remaps=[("request.firstline.uri.query.g", "HTTP.URI"), ("request.firstline.uri.query.r", "HTTP.URI"),
                 ("request.firstline.uri.query.s", "SCREENRESOLUTION")],
         skipped=["SCREENWIDTH / SCREENHEIGHT (the example's own ScreenResolutionDissector)", "GeoIP fields"])

# --------------------------------------------------------------------- NGINX
# hpt/nginxmodules/NginxUpstreamTest.java:49-90 (testBasicLogFormat)
UP_ADDR = "192.168.1.1:80, 192.168.1.2:80, unix:/tmp/sock : 192.168.10.1:80, 192.168.10.2:80"
UP_NUM = "1, 2, 3 : 4, 5"
UP_TIME = "1.001, 2.002, 3.003 : 4.004, 5.005"
UP_STATUS = "111, 222, 333 : 444, 555"


def up_expect(typ, base, vals):
    """N.value / N.redirected for the 4 servers of the lists above + absent N=4"""
    e, a = {}, []
    for k, (v, r) in enumerate(vals):
        e["%s:%s.%d.value" % (typ, base, k)] = v
        e["%s:%s.%d.redirected" % (typ, base, k)] = r
    a = ["%s:%s.4.value" % (typ, base), "%s:%s.4.redirected" % (typ, base)]
    return e, a


e1, a1 = up_expect("UPSTREAM_ADDR", "nginxmodule.upstream.addr",
                   [("192.168.1.1:80",) * 2, ("192.168.1.2:80",) * 2, ("unix:/tmp/sock", "192.168.10.1:80"),
                    ("192.168.10.2:80",) * 2])
e2, a2 = up_expect("BYTES", "nginxmodule.upstream.bytes.received", [("1", "1"), ("2", "2"), ("3", "4"), ("5", "5")])
e1.update(e2)
e1["UPSTREAM_ADDR_LIST:nginxmodule.upstream.addr"] = UP_ADDR
e1["UPSTREAM_BYTES_LIST:nginxmodule.upstream.bytes.received"] = UP_NUM
case("hpt/nginxmodules/NginxUpstreamTest.java:49-90", "\"$upstream_addr\" \"$upstream_bytes_received\"",
     "\"%s\" \"%s\"" % (UP_ADDR, UP_NUM), list(e1) + a1 + a2, expect=e1, absent=a1 + a2)

# hpt/nginxmodules/NginxUpstreamTest.java:93-113 (testFullLine; config 4's log_format)
NGINX_CFG4 = ("$remote_addr - $remote_user [$time_local] \"$request\" $status $body_bytes_sent \"$http_referer\" "
              "\"$http_user_agent\" \"$http_x_forwarded_for\" $request_time $upstream_response_time $pipe")
UPR = "nginxmodule.upstream.response.time"
case("hpt/nginxmodules/NginxUpstreamTest.java:93-113", NGINX_CFG4,
     "10.77.150.123 - - [15/Dec/2018:19:27:57 -0500] \"GET /25.chunk.js HTTP/1.1\" 200 84210 "
     "\"https://api.demo.com/\" \"Mozilla/5.0 (Windows NT 10.0; Win64; x64) AppleWebKit/537.36 (KHTML, like Gecko) "
     "Chrome/70.0.3538.110 Safari/537.36\" \"-\" 0.002 0.002 .",
     ["SECOND_MILLIS:%s.0.value" % UPR, "SECOND_MILLIS:%s.0.redirected" % UPR,
      "MICROSECONDS:%s.0.value" % UPR, "MICROSECONDS:%s.0.redirected" % UPR],
     expect={"SECOND_MILLIS:%s.0.value" % UPR: "0.002", "SECOND_MILLIS:%s.0.redirected" % UPR: "0.002",
             "MICROSECONDS:%s.0.value" % UPR: {"l": 2000}, "MICROSECONDS:%s.0.redirected" % UPR: {"l": 2000}})

# hpt/nginxmodules/NginxUpstreamTest.java:116-267 (validateAllFields): one-variable formats
UPS = [("$upstream_addr", UP_ADDR, "UPSTREAM_ADDR", "nginxmodule.upstream.addr",
        [("192.168.1.1:80",) * 2, ("192.168.1.2:80",) * 2, ("unix:/tmp/sock", "192.168.10.1:80"), ("192.168.10.2:80",) * 2])]
for var, base in [("$upstream_bytes_received", "bytes.received"), ("$upstream_bytes_sent", "bytes.sent"),
                  ("$upstream_response_length", "response.length")]:
    UPS.append((var, UP_NUM, "BYTES", "nginxmodule.upstream." + base, [("1", "1"), ("2", "2"), ("3", "4"), ("5", "5")]))
for var, base in [("$upstream_connect_time", "connect.time"), ("$upstream_header_time", "header.time"),
                  ("$upstream_queue_time", "queue.time"), ("$upstream_response_time", "response.time"),
                  ("$upstream_first_byte_time", "first_byte.time"), ("$upstream_session_time", "session.time")]:
    UPS.append((var, UP_TIME, "SECOND_MILLIS", "nginxmodule.upstream." + base,
                [("1.001", "1.001"), ("2.002", "2.002"), ("3.003", "4.004"), ("5.005", "5.005")]))
UPS.append(("$upstream_status", UP_STATUS, "UPSTREAM_STATUS", "nginxmodule.upstream.status",
            [("111", "111"), ("222", "222"), ("333", "444"), ("555", "555")]))
for var, line, typ, base, vals in UPS:
    e, a = up_expect(typ, base, vals)
    case("hpt/nginxmodules/NginxUpstreamTest.java:116-267", var, line, list(e) + a, expect=e, absent=a)
for var, line, field in [("$upstream_cache_status", "STALE", "UPSTREAM_CACHE_STATUS:nginxmodule.upstream.cache.status"),
                         ("$upstream_cookie_mycookie", "MyValue", "HTTP.COOKIE:nginxmodule.upstream.response.cookies.mycookie"),
                         ("$upstream_http_myheader", "MyValue", "HTTP.HEADER:nginxmodule.upstream.header.myheader"),
                         ("$upstream_trailer_mytrailer", "MyValue", "HTTP.TRAILER:nginxmodule.upstream.trailer.mytrailer")]:
    case("hpt/nginxmodules/NginxUpstreamTest.java:116-267", var, line, [field], expect={field: line})

# hpt/NginxLogFormatTest.java:78-92 (unknown variables)
case("hpt/NginxLogFormatTest.java:78-92",
     "$foobar $remote_user_age $remote_addr - $remote_user [$time_local] \"$request\" $status $body_bytes_sent "
     "\"$http_referer\" \"$http_user_agent\"",
     "something 42 123.65.150.10 - - [23/Aug/2010:03:50:59 +0000] \"POST /wordpress3/wp-admin/admin-ajax.php HTTP/1.1\" "
     "200 2 \"http://www.example.com/wordpress3/wp-admin/post-new.php\" \"Mozilla/5.0 (Macintosh; U; Intel Mac OS X "
     "10_6_4; en-US) AppleWebKit/534.3 (KHTML, like Gecko) Chrome/6.0.472.25 Safari/534.3\"",
     ["UNKNOWN_NGINX_VARIABLE:nginx.unknown.foobar", "UNKNOWN_NGINX_VARIABLE:nginx.unknown.remote_user_age"],
     expect={"UNKNOWN_NGINX_VARIABLE:nginx.unknown.foobar": "something",
             "UNKNOWN_NGINX_VARIABLE:nginx.unknown.remote_user_age": "42"})

# hpt/NginxLogFormatTest.java:347-425 (validateAllFields): (format, line, field, value); long-valued
# outputs of the converters and the timestamp dissector are {"l": n} in the canonical record
NGINX_FIELDS = [
    ("$status", "200", "STRING:request.status.last", "200"),
    ("$time_iso8601", "2017-01-03T15:56:36+01:00", "TIME.ISO8601:request.receive.time", "2017-01-03T15:56:36+01:00"),
    ("$time_local", "03/Jan/2017:15:56:36 +0100", "TIME.STAMP:request.receive.time", "03/Jan/2017:15:56:36 +0100"),
    ("$time_local", "03/Jan/2017:15:56:36 +0100", "TIME.EPOCH:request.receive.time.epoch", {"l": 1483455396000}),
    ("$msec", "1483455396.639", "TIME.EPOCH:request.receive.time.epoch", {"l": 1483455396639}),
    ("$remote_addr", "127.0.0.1", "IP:connection.client.host", "127.0.0.1"),
    ("$binary_remote_addr", "\\x7F\\x00\\x00\\x01", "IP_BINARY:connection.client.host", "\\x7F\\x00\\x00\\x01"),
    ("$binary_remote_addr", "\\x7F\\x00\\x00\\x01", "IP:connection.client.host", "127.0.0.1"),
    ("$remote_port", "44448", "PORT:connection.client.port", "44448"),
    ("$remote_user", "-", "STRING:connection.client.user", None),
    ("$is_args", "?", "STRING:request.firstline.uri.is_args", "?"),
    ("$query_string", "aap&noot=&mies=wim", "HTTP.QUERYSTRING:request.firstline.uri.query", "aap&noot=&mies=wim"),
    ("$args", "aap&noot=&mies=wim", "HTTP.QUERYSTRING:request.firstline.uri.query", "aap&noot=&mies=wim"),
    ("$args", "aap&noot=&mies=wim", "STRING:request.firstline.uri.query.aap", ""),
    ("$args", "aap&noot=&mies=wim", "STRING:request.firstline.uri.query.noot", ""),
    ("$args", "aap&noot=&mies=wim", "STRING:request.firstline.uri.query.mies", "wim"),
    ("$arg_name", "foo", "STRING:request.firstline.uri.query.name", "foo"),
    ("$bytes_sent", "694", "BYTES:response.bytes", "694"),
    ("$bytes_received", "694", "BYTES:request.bytes", "694"),
    ("$body_bytes_sent", "436", "BYTES:response.body.bytes", "436"),
    ("$connection", "5", "NUMBER:connection.serial_number", "5"),
    ("$connection_requests", "4", "NUMBER:connection.requestnr", "4"),
    ("$https", "", "STRING:connection.https", ""),
    ("$content_length", "-", "HTTP.HEADER:request.header.content_length", None),
    ("$content_type", "-", "HTTP.HEADER:request.header.content_type", None),
    ("$cookie_name", "Something", "HTTP.COOKIE:request.cookies.name", "Something"),
    ("$document_root", "/var/www/html", "STRING:request.firstline.document_root", "/var/www/html"),
    ("$realpath_root", "/var/www/html", "STRING:request.firstline.realpath_root", "/var/www/html"),
    ("$host", "localhost", "STRING:connection.server.name", "localhost"),
    ("$hostname", "hackbox", "STRING:connection.client.host", "hackbox"),
    ("$http_foobar", "Something", "HTTP.HEADER:request.header.foobar", "Something"),
    ("$sent_http_foobar", "Something", "HTTP.HEADER:response.header.foobar", "Something"),
    ("$sent_trailer_foobar", "Something", "HTTP.TRAILER:response.trailer.foobar", "Something"),
    ("$nginx_version", "1.10.0", "STRING:server.nginx.version", "1.10.0"),
    ("$pid", "5137", "NUMBER:connection.server.child.processid", "5137"),
    ("$pipe", ".", "STRING:connection.nginx.pipe", "."),
    ("$pipe", "p", "STRING:connection.nginx.pipe", "p"),
    ("$protocol", "TCP", "STRING:connection.protocol", "TCP"),
    ("$proxy_protocol_addr", "1.2.3.4", "IP:connection.client.proxy.host", "1.2.3.4"),
    ("$proxy_protocol_port", "1234", "PORT:connection.client.proxy.port", "1234"),
    ("$request", "GET /?aap&noot=&mies=wim HTTP/1.1", "HTTP.FIRSTLINE:request.firstline", "GET /?aap&noot=&mies=wim HTTP/1.1"),
    ("$request_completion", "OK", "STRING:request.completion", "OK"),
    ("$request_filename", "/var/www/html/index.html", "FILENAME:server.filename", "/var/www/html/index.html"),
    ("$request_length", "491", "BYTES:request.bytes", "491"),
    ("$request_method", "GET", "HTTP.METHOD:request.firstline.method", "GET"),
    ("$request_time", "123.456", "SECOND_MILLIS:response.server.processing.time", "123.456"),
    ("$request_time", "123.456", "MILLISECONDS:response.server.processing.time", {"l": 123456}),
    ("$request_time", "123.456", "MICROSECONDS:response.server.processing.time", {"l": 123456000}),
    ("$request_uri", "/?aap&noot=&mies=wim", "HTTP.URI:request.firstline.uri", "/?aap&noot=&mies=wim"),
    ("$scheme", "http", "HTTP.PROTOCOL:request.firstline.uri.protocol", "http"),
    ("$sent_http_etag", "W/\\x22586bbb8b-29e\\x22", "HTTP.HEADER:response.header.etag", "W/\\x22586bbb8b-29e\\x22"),
    ("$sent_http_last_modified", "Tue, 03 Jan 2017 14:56:11 GMT", "HTTP.HEADER:response.header.last_modified",
     "Tue, 03 Jan 2017 14:56:11 GMT"),
    ("$server_addr", "127.0.0.1", "IP:connection.server.ip", "127.0.0.1"),
    ("$server_name", "_", "STRING:connection.server.name", "_"),
    ("$server_port", "80", "PORT:connection.server.port", "80"),
    ("$server_protocol", "HTTP/1.1", "HTTP.PROTOCOL_VERSION:request.firstline.protocol", "HTTP/1.1"),
    ("$server_protocol", "HTTP/1.1", "HTTP.PROTOCOL:request.firstline.protocol", "HTTP"),
    ("$server_protocol", "HTTP/1.1", "HTTP.PROTOCOL.VERSION:request.firstline.protocol.version", "1.1"),
    ("$tcpinfo_rtt", "52", "MICROSECONDS:connection.tcpinfo.rtt", "52"),
    ("$tcpinfo_rttvar", "30", "MICROSECONDS:connection.tcpinfo.rttvar", "30"),
    ("$tcpinfo_snd_cwnd", "10", "BYTES:connection.tcpinfo.send.cwnd", "10"),
    ("$tcpinfo_rcv_space", "43690", "BYTES:connection.tcpinfo.receive.space", "43690"),
    ("$uri", "/index.html", "HTTP.URI:request.firstline.uri.normalized", "/index.html"),
    ("$document_uri", "/index.html", "HTTP.URI:request.firstline.uri.normalized", "/index.html"),
    ("$http_user_agent", "Mozilla/5.0 (Foo)", "HTTP.USERAGENT:request.user-agent", "Mozilla/5.0 (Foo)"),
    ("$http_foo_user_agent", "Mozilla/5.0 (Foo)", "HTTP.HEADER:request.header.foo_user_agent", "Mozilla/5.0 (Foo)"),
    ("$http_user_agent_foo", "Mozilla/5.0 (Foo)", "HTTP.HEADER:request.header.user_agent_foo", "Mozilla/5.0 (Foo)"),
    ("$http_referer", "http://localhost/", "HTTP.URI:request.referer", "http://localhost/"),
    ("$request_body", "-", "NOT_IMPLEMENTED:nginx_parameter_not_intended_for_logging__request_body", None),
    ("$request_body_file", "-", "NOT_IMPLEMENTED:nginx_parameter_not_intended_for_logging__request_body_file", None),
    ("$limit_rate", "0", "NOT_IMPLEMENTED:nginx_parameter_not_intended_for_logging__limit_rate", "0"),
]
for fmt, line, field, want in NGINX_FIELDS:
    case("hpt/NginxLogFormatTest.java:347-425", fmt, line, [field], expect={field: want})
# (:350 $time_iso8601 -> TIME.EPOCH goes through TimeStampDissector("TIME.ISO8601"), not restated: left out)

# resilientUrlDecode (hpt/UtilsTest.java:27-49): unit vectors, not whole lines
URLDECODE = [
    ["  ", "  "], [" %20", "  "], ["%20 ", "  "], ["%20%20", "  "], ["%u0020%u0020", "  "], ["%20%u0020", "  "],
    ["%u0020%20", "  "], ["x %2", "x "], ["x%20%2", "x "], ["x%u202", "x"], ["x%u20", "x"], ["x%u2", "x"],
    ["x%u", "x"], ["x%", "x"], ["%20 %20%u0020%20 %20%2", "       "],
]

# Setup-time failures (the parser refuses the requested paths before any line
# is parsed): MissingDissectorsException with the offending path, lower-cased
# as the reference reports it.
SETUP = [
    {"source": "hpt/ApacheHttpdLogParserTest.java:242-259 (testMissing)", "logformat": FULLCOMBINED,
     "fields": ["STRING:request.firstline.uri.query.ThisShouldNOTBeMissing",
                "HEADER:response.header.Etag.ThisShouldBeMissing"],
     "error": "MissingDissectorsException", "message_contains": "HEADER:response.header.etag.thisshouldbemissing"},
    {"source": "hpt/ApacheHttpdLogParserTest.java:263-279 (testMissing2)", "logformat": FULLCOMBINED,
     "fields": ["BLURP:request.firstline.uri.query.ThisShouldBeMissing", "HTTP.HEADER:response.header.etag"],
     "error": "MissingDissectorsException", "message_contains": "BLURP:request.firstline.uri.query.thisshouldbemissing"},
    {"source": "hpt/ApacheHttpdLogParserTest.java:472-485 (testFailOnMissingDissectors)", "logformat": "%t",
     "fields": ["STRING:request.firstline.uri.query.foo", "TIME.EPOCH:request.receive.time.epoch"],
     "error": "MissingDissectorsException", "message_contains": "STRING:request.firstline.uri.query.foo"},
]

if __name__ == "__main__":
    out = {"generated_by": "tests/golden/make_golden.py", "cases": CASES, "setup_cases": SETUP,
           "url_decode": {"source": "hpt/UtilsTest.java:27-49", "vectors": URLDECODE}}
    with open(os.path.join(HERE, "reference_vectors.json"), "w", encoding="utf-8") as f:
        json.dump(out, f, indent=1, ensure_ascii=False)
    print("wrote", len(CASES), "cases")
