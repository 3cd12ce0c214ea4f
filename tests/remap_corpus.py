"""Type-remapping test corpus (Parser.addTypeRemapping, core/Parser.java:
636-677; Parsable.addDissection, core/Parsable.java:160-176): 'combined' lines
whose request carries URLs inside query parameters (percent-encoded or plain,
with queries, fragments, ports, userinfo, nested encoded URLs, repeated and
empty parameters) and whose user agent is sometimes a URL, parsed with those
parameters / the user agent remapped to HTTP.URI.  Shared by the CPU
(emulated) and GPU parity tests; the oracle decides every line."""
import random
import urllib.parse

FORMAT = "combined"
REMAPS = [("request.firstline.uri.query.url", "HTTP.URI"),
          ("request.firstline.uri.query.url.query.next", "HTTP.URI"),
          ("request.referer.query.u", "HTTP.URI"),
          ("request.user-agent", "HTTP.URI"),
          ("request.firstline.uri.query.tag", "SOMETAG")]
_U = "request.firstline.uri.query.url"
FIELDS = ["HTTP.URI:" + _U, "STRING:" + _U, "HTTP.HOST:%s.host" % _U, "HTTP.PORT:%s.port" % _U,
          "HTTP.PATH:%s.path" % _U, "HTTP.QUERYSTRING:%s.query" % _U, "HTTP.REF:%s.ref" % _U,
          "HTTP.PROTOCOL:%s.protocol" % _U, "HTTP.USERINFO:%s.userinfo" % _U, "STRING:%s.query.*" % _U,
          "HTTP.HOST:%s.query.next.host" % _U, "STRING:%s.query.next.query.id" % _U,
          "HTTP.HOST:request.referer.query.u.host", "STRING:request.referer.query.u.query.q",
          "HTTP.HOST:request.user-agent.host", "HTTP.PATH:request.user-agent.path",
          "SOMETAG:request.firstline.uri.query.tag", "STRING:request.firstline.uri.query.a",
          "HTTP.PATH:request.firstline.uri.path", "IP:connection.client.host"]

HOSTS = ["www.example.com", "shop.example.nl", "10.1.2.3", "localhost", "a-b.c-d.org", "x.y", "[::1]"]
PATHS = ["/", "/a/b/c.html", "/search", "/p/123/", "/%7Euser/index.php", "/with space", "/ümlaut"]


def _inner(rng, depth=0):
    if rng.random() < 0.75:  # the common shape: no userinfo / IPv6 / odd fragments
        host = rng.choice(HOSTS[:5])
        url = "%s://%s%s%s" % (rng.choice(["http", "https"]), host, rng.choice(["", "", ":8080"]),
                               rng.choice(PATHS[:4]))
        if rng.random() < 0.7:
            parts = ["id=%d" % rng.randrange(1000), "q=" + rng.choice(["a+b", "x%20y", "plain", ""]),
                     "promo=koken-pannen_%d" % rng.randrange(999)]
            if depth == 0 and rng.random() < 0.4:
                parts.append("next=" + urllib.parse.quote(_inner(rng, 1), safe=""))
            url += "?" + "&".join(rng.sample(parts, rng.randint(1, len(parts))))
        return url + rng.choice(["", "", "#top"])
    scheme = rng.choice(["http", "https", "ftp", "HTTP"])
    host = rng.choice(HOSTS)
    port = rng.choice(["", "", ":8080", ":0", ":99999999999"])
    ui = rng.choice(["", "", "", "user:pw@"])
    path = rng.choice(PATHS)
    q = ""
    if rng.random() < 0.7:
        parts = ["id=%d" % rng.randrange(1000), "q=" + rng.choice(["a+b", "x%20y", "%E2%82%AC", "plain", ""]),
                 rng.choice(["promo=koken", "Upper=Case", "a=1&a=2", "e", "x=%zz"])]
        if depth == 0 and rng.random() < 0.4:
            parts.append("next=" + urllib.parse.quote(_inner(rng, 1), safe=""))
        q = "?" + "&".join(rng.sample(parts, rng.randint(1, len(parts))))
    frag = rng.choice(["", "", "#top", "#a%20b", "#x?y"])
    if rng.random() < 0.15:
        return rng.choice(["/relative/path?x=1", "mailto:someone@example.com", "just-text", "//host.only/p",
                           "http://", "http://host:port/", "%", "http://h/p#f#g"])
    return "%s://%s%s%s%s%s%s" % (scheme, ui, host, port, path, q, frag)


def _enc(rng, s):
    r = rng.random()
    if r < 0.65:
        return urllib.parse.quote(s, safe="")
    if r < 0.75:
        return urllib.parse.quote_plus(s, safe=":/")
    if r < 0.95:  # plain: only the bytes a query piece cannot hold are escaped
        return s.replace("&", "%26").replace("#", "%23").replace(" ", "+")
    return urllib.parse.quote(s, safe="") + rng.choice(["%", "%4", "%zz"])  # broken escapes


def line(rng, k):
    params = []
    n_url = rng.choice([0] + [1] * 8 + [2])
    for _ in range(n_url):
        params.append("url=" + (_enc(rng, _inner(rng)) if rng.random() < 0.95 else ""))
    if rng.random() < 0.5:
        params.append("a=" + rng.choice(["1", "x%2By", "%41"]))
    if rng.random() < 0.3:
        params.append("tag=" + rng.choice(["t1", "t%202", ""]))
    rng.shuffle(params)
    req = "/page" + ("?" + "&".join(params) if params else "")
    ref = "-"
    if rng.random() < 0.6:
        ref = "http://ref.example.com/r?u=%s&z=1" % _enc(rng, _inner(rng))
    ua = rng.choice(["Mozilla/5.0 (X11; Linux x86_64)", _inner(rng), "curl/8.0", "http://bot.example.com/info?x=1",
                     "Mozilla/5.0 (compatible; Bot/2.1; +http://www.example.com/bot.html)"])
    return ('10.0.%d.%d - - [10/Oct/2020:13:55:36 +0200] "GET %s HTTP/1.1" 200 %d "%s" "%s"'
            % (k % 250, (k // 250) % 250, req, rng.randrange(1, 99999), ref, ua)).encode("utf-8")


def corpus(seed, n):
    rng = random.Random(seed)
    return [line(rng, k) for k in range(n)]
