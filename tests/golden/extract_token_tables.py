#!/usr/bin/env python3
"""Extract the LogFormat token tables from the reference's Java sources into
tests/golden/token_tables.json.

The planner (logparser_amd/csrc/plan.cpp apache_table()/nginx_table()) and
the CPU oracle (oracle/oracle.c apache_token_parsers()/nginx_token_parsers())
each carry a hand transcription of these tables.  This script derives them a
third way -- by reading the reference's Java text, with no transcription in
between -- so the tests can check both transcriptions against it
(tests/test_token_tables.py).

Only the reference's text is read; nothing is compiled or run.  A small
evaluator understands the statement shapes the tables are written in:

  ApacheHttpdLogFormatDissector.createAllTokenParsers  (:199-638)
    parsers.add(new FixedStringTokenParser(tok, regex))
    parsers.add(new NamedTokenParser(pattern, name, type, casts, regex[, prio]))
    parsers.add(new ParameterizedTokenParser(pattern, name, type, casts, regex, prio, new X()))
    parsers.addAll(createFirstAndLastTokenParsers(tok, name, type, casts, regex[, prio]))
    addExtraOutput(parsers, tok, new TokenOutputField(type, name, casts)[.deprecateFor(..)])
  nginxmodules/*Module.getTokenParsers, in NginxHttpdLogFormatDissector's module order (:121-131)
    parsers.add(new TokenParser(tok, name, type, casts, regex[, prio]))
    parsers.add(new NamedTokenParser(...))
    parsers.add(new TokenFormatDissector.NotImplementedTokenParser(tok, prefix[, regex], prio))

String constants (TokenParser.FORMAT_*, HttpFirstLineDissector.FIRSTLINE_REGEX,
module PREFIX), the Casts sets (core/Casts.java) and one-line helper methods
(UpstreamModule.upstreamListOf) are evaluated from their own source text.
The semantics applied by the constructors are restated with citations:
default priorities (TokenParser.java:77-83 -> 10, NamedTokenParser.java:34-41
-> 0, FixedStringTokenParser -> 0), TokenOutputField lowercasing the name
(TokenOutputField.java:39-44), NotImplementedTokenParser's output name
(TokenFormatDissector.java:89-103), createFirstAndLastTokenParsers' expansion
(ApacheHttpdLogFormatDissector.java:651-714; the "original" token list is read
from its case labels) and addExtraOutput (:640-649).

usage: python3 tests/golden/extract_token_tables.py [REFERENCE_ROOT] [OUT_JSON]
"""
import hashlib
import json
import os
import re
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
OUT = os.path.join(HERE, "token_tables.json")
HP = "httpdlog/httpdlog-parser/src/main/java/nl/basjes/parse/httpdlog"
CASTS = "parser-core/src/main/java/nl/basjes/parse/core/Casts.java"
APACHE = HP + "/ApacheHttpdLogFormatDissector.java"
NGINX = HP + "/NginxHttpdLogFormatDissector.java"
TOKENPARSER = HP + "/dissectors/tokenformat/TokenParser.java"
FIRSTLINE = HP + "/dissectors/HttpFirstLineDissector.java"
MODULES = HP + "/dissectors/nginxmodules/"


# ------------------------------------------------------------------ lexer
TOK_RE = re.compile(r"""
    (?P<ws>\s+)
  | (?P<lc>//[^\n]*)
  | (?P<bc>/\*.*?\*/)
  | (?P<str>"(?:[^"\\]|\\.)*")
  | (?P<chr>'(?:[^'\\]|\\.)*')
  | (?P<num>\d+)
  | (?P<id>[A-Za-z_$][A-Za-z_0-9$]*)
  | (?P<op>::|->|[-+*/%=<>!&|?:;,.(){}\[\]@^~])
""", re.S | re.X)

ESC = {"n": "\n", "t": "\t", "r": "\r", "b": "\b", "f": "\f", "0": "\0", "\\": "\\", '"': '"', "'": "'"}


def unescape(body):
    out, i = [], 0
    while i < len(body):
        c = body[i]
        if c != "\\":
            out.append(c)
            i += 1
            continue
        n = body[i + 1]
        if n == "u":
            out.append(chr(int(body[i + 2:i + 6], 16)))
            i += 6
        else:
            out.append(ESC[n])
            i += 2
    return "".join(out)


def lex(text):
    toks, pos = [], 0
    while pos < len(text):
        m = TOK_RE.match(text, pos)
        if not m:
            raise SyntaxError("cannot lex at %r" % text[pos:pos + 40])
        pos = m.end()
        k = m.lastgroup
        if k in ("ws", "lc", "bc"):
            continue
        v = m.group()
        if k == "str":
            toks.append(("str", unescape(v[1:-1])))
        elif k == "num":
            toks.append(("num", int(v)))
        else:
            toks.append((k, v))
    return toks


# --------------------------------------------------------------- sources
class Src:
    def __init__(self, root, rel):
        self.rel = rel
        with open(os.path.join(root, rel), "rb") as f:
            raw = f.read()
        self.sha256 = hashlib.sha256(raw).hexdigest()
        self.toks = lex(raw.decode("utf-8"))

    def method_body(self, name):
        """tokens between the braces of the (last-declared) method `name` with a body"""
        t = self.toks
        found = None
        for i in range(len(t) - 1):
            if t[i] == ("id", name) and t[i + 1] == ("op", "(") and i > 0 and is_decl(t[i - 1]):
                j = match(t, i + 1)
                if j + 1 < len(t) and t[j + 1] == ("op", "{"):
                    found = (i, j + 1)
        if not found:
            raise LookupError("%s: method %s not found" % (self.rel, name))
        i, b = found
        return t[i + 2:match(t, i + 1)], t[b + 1:match(t, b)]

    def methods(self, name):
        """every (params, body) overload of method `name`"""
        t, res = self.toks, []
        for i in range(1, len(t) - 1):
            if t[i] == ("id", name) and t[i + 1] == ("op", "(") and i > 0 and is_decl(t[i - 1]):
                j = match(t, i + 1)
                if j + 1 < len(t) and t[j + 1] == ("op", "{"):
                    res.append((t[i + 2:j], t[j + 2:match(t, j + 1)]))
        return res


def is_decl(prev):
    """the token before a method name in a declaration: its return type"""
    return prev == ("op", ">") or (prev[0] == "id" and prev[1] not in ("new", "return"))


def match(t, i):
    """index of the bracket closing the one at t[i]"""
    pairs = {"(": ")", "{": "}", "[": "]"}
    o = t[i][1]
    c = pairs[o]
    d = 0
    for j in range(i, len(t)):
        if t[j] == ("op", o):
            d += 1
        elif t[j] == ("op", c):
            d -= 1
            if d == 0:
                return j
    raise SyntaxError("unbalanced %s" % o)


def split_top(t, sep):
    parts, cur, d = [], [], 0
    for x in t:
        if x[0] == "op" and x[1] in "({[":
            d += 1
        elif x[0] == "op" and x[1] in ")}]":
            d -= 1
        if d == 0 and x == ("op", sep):
            parts.append(cur)
            cur = []
        else:
            cur.append(x)
    if cur:
        parts.append(cur)
    return parts


# --------------------------------------------------------------- values
class Parser:
    """A TokenParser under construction (kind, token, regex, prio, custom, outs)."""

    def __init__(self, kind, token, regex, prio, custom=None):
        self.kind, self.token, self.regex, self.prio, self.custom = kind, token, regex, prio, custom
        self.outs = []

    def add_out(self, typ, name, casts):
        # TokenOutputField lowercases the name (TokenOutputField.java:39-44)
        self.outs.append([typ, name.lower(), list(casts)])
        return self

    def json(self):
        return {"kind": self.kind, "token": self.token, "regex": self.regex, "prio": self.prio,
                "custom": self.custom, "outs": self.outs}


class Out:
    def __init__(self, typ, name, casts):
        self.typ, self.name, self.casts = typ, name, casts


class Obj:
    def __init__(self, cls):
        self.cls = cls


class Casts(tuple):
    pass


class Env:
    def __init__(self, consts, funcs, fl_original):
        self.consts = consts          # name -> value
        self.funcs = funcs            # name -> (param names, return expr tokens)
        self.fl_original = fl_original

    # expr := term ('+' term)*
    def expr(self, t):
        v, i = self.term(t, 0)
        while i < len(t):
            if t[i] != ("op", "+"):
                raise SyntaxError("unexpected %r" % (t[i],))
            w, i = self.term(t, i + 1)
            v = v + w if isinstance(v, str) else (v + w)
        return v

    def args(self, t, i):
        j = match(t, i)
        return [self.expr(a) for a in split_top(t[i + 1:j], ",")], j + 1

    def term(self, t, i):
        if t[i] == ("op", "-"):
            v, i = self.term(t, i + 1)
            return -v, i
        if t[i] == ("op", "("):
            j = match(t, i)
            return self.expr(t[i + 1:j]), j + 1
        k, v = t[i]
        if k in ("str", "num"):
            val, i = v, i + 1
        elif v == "new":
            name, i = self.qual(t, i + 1)
            if t[i] == ("op", "<"):  # generics: new ArrayList<>(...)
                while t[i] != ("op", ">"):
                    i += 1
                i += 1
            args, i = self.args(t, i)
            val = self.construct(name[-1], args)
        elif k == "id":
            name, i = self.qual(t, i)
            if i < len(t) and t[i] == ("op", "("):
                args, i = self.args(t, i)
                val = self.call(name, args)
            else:
                val = self.const(name[-1])
        else:
            raise SyntaxError("unexpected %r" % (t[i],))
        while i < len(t) and t[i] == ("op", "."):  # method chains
            m = t[i + 1][1]
            args, i = self.args(t, i + 2)
            val = self.chain(val, m, args)
        return val, i

    @staticmethod
    def qual(t, i):
        name = [t[i][1]]
        i += 1
        while i + 1 < len(t) and t[i] == ("op", ".") and t[i + 1][0] == "id":
            name.append(t[i + 1][1])
            i += 2
        return name, i

    def const(self, n):
        if n not in self.consts:
            raise LookupError("unknown constant " + n)
        return self.consts[n]

    def call(self, name, args):
        n = name[-1]
        if n == "of" and name[0] == "EnumSet":
            return Casts(sorted(args, key=self.CAST_ORDER.index))  # EnumSet iterates in declaration order
        if n == "noneOf":
            return Casts(())
        if n == "createFirstAndLastTokenParsers":
            return self.first_last(*args)
        if n in self.funcs:
            params, body = self.funcs[n]
            sub = Env(dict(self.consts, **dict(zip(params, args))), self.funcs, self.fl_original)
            return sub.expr(body)
        raise LookupError("unknown call " + ".".join(name))

    def construct(self, cls, a):
        if cls == "FixedStringTokenParser":  # TokenFormatDissector.java:61-63: prio 0
            return Parser("fixed", a[0], a[1], 0)
        if cls == "TokenParser":
            if len(a) in (5, 6, 7):       # TokenParser.java:77-106: default prio 10
                p = Parser("plain", a[0], a[4], a[5] if len(a) > 5 else 10)
                return p.add_out(a[2], a[1], a[3])
            if len(a) in (2, 3):          # TokenParser.java:108-117: no outputs, default prio 0
                return Parser("plain", a[0], a[1], a[2] if len(a) > 2 else 0)
        if cls == "NamedTokenParser":     # NamedTokenParser.java:34-41: default prio 0
            return Parser("named", a[0], a[4], a[5] if len(a) > 5 else 0).add_out(a[2], a[1], a[3])
        if cls == "ParameterizedTokenParser":
            custom = a[6].cls if len(a) > 6 and isinstance(a[6], Obj) else None
            return Parser("param", a[0], a[4], a[5], custom).add_out(a[2], a[1], a[3])
        if cls == "NotImplementedTokenParser":  # TokenFormatDissector.java:89-103
            tok, prefix = a[0], a[1]
            regex, prio = (a[2], a[3]) if len(a) == 4 else (".*", a[2])
            name = prefix + "_" + re.sub(r"[^a-z0-9_]", "_", tok.lower())
            return Parser("plain", tok, regex, prio).add_out("NOT_IMPLEMENTED", name, ("STRING",))
        if cls == "TokenOutputField":
            return Out(a[0], a[1], a[2])
        if cls == "ArrayList":
            return []
        return Obj(cls)

    @staticmethod
    def chain(val, m, args):
        if m == "addOutputField" and isinstance(val, Parser):
            return val.add_out(args[0], args[1], args[2])
        if m in ("setWarningMessageWhenUsed", "deprecateFor"):
            return val
        if m == "replaceFirst" and isinstance(val, str):
            return val.replace(args[0], args[1], 1)
        raise LookupError("unknown method ." + m)

    def first_last(self, tok, name, typ, casts, regex, prio=0):
        # ApacheHttpdLogFormatDissector.createFirstAndLastTokenParsers (:651-714)
        a = Parser("plain", tok, regex, prio).add_out(typ, name, casts)
        a.add_out(typ, name + (".original" if tok in self.fl_original else ".last"), casts)
        b = Parser("plain", tok.replace("%", "%<", 1), regex, prio).add_out(typ, name + ".original", casts)
        c = Parser("plain", tok.replace("%", "%>", 1), regex, prio).add_out(typ, name + ".last", casts)
        return [a, b, c]


def string_constants(src, into, env):
    """evaluate every `static final String NAME = expr;` of a file in order"""
    t = src.toks
    for i in range(len(t) - 4):
        if t[i] == ("id", "final") and t[i + 1] == ("id", "String") and t[i + 2][0] == "id" \
                and t[i + 3] == ("op", "=") and t[i - 1] == ("id", "static"):
            j = i + 4
            d = 0
            while not (d == 0 and t[j] == ("op", ";")):
                d += t[j] in (("op", "("),) and 1 or 0
                d -= t[j] in (("op", ")"),) and 1 or 0
                j += 1
            into[t[i + 2][1]] = env.expr(t[i + 4:j])


def casts_constants(src, into, env):
    t = src.toks
    # the enum's members, in declaration order: `enum Casts { STRING, LONG, DOUBLE; ...`
    i = t.index(("id", "enum"))
    j = t.index(("op", ";"), i)
    members = [x[1] for x in t[i + 3:j] if x[0] == "id"]
    Env.CAST_ORDER = members
    into.update({m: m for m in members})
    into["class"] = None  # EnumSet.noneOf(Casts.class)
    for i in range(len(t) - 4):
        if t[i] == ("id", "EnumSet") and t[i + 1] == ("op", "<") and t[i + 4][0] == "id" \
                and t[i + 5] == ("op", "="):
            j = i + 6
            while t[j] != ("op", ";"):
                j += 1
            into[t[i + 4][1]] = env.expr(t[i + 6:j])


def helper_funcs(src):
    """private one-statement helpers `T f(String a, ...) { return expr; }`"""
    out = {}
    t = src.toks
    for i in range(1, len(t) - 1):
        if t[i][0] == "id" and t[i + 1] == ("op", "(") and t[i - 1] == ("id", "String"):
            j = match(t, i + 1)
            if j + 2 < len(t) and t[j + 1] == ("op", "{") and t[j + 2] == ("id", "return"):
                params = [p[-1][1] for p in split_top(t[i + 2:j], ",")]
                e = j + 3
                while t[e] != ("op", ";"):
                    e += 1
                out[t[i][1]] = (params, t[j + 3:e])
    return out


def run_body(body, env, parsers):
    for st in split_top(body, ";"):
        if not st:
            continue
        if st[0] == ("id", "List") or st[0] == ("id", "return"):
            continue  # `List<TokenParser> parsers = new ArrayList<>(..)`, `return parsers`
        if st[0] == ("id", "final"):
            st = st[1:]
        if st[0] == ("id", "String") and st[2] == ("op", "="):  # local `String x = expr`
            env.consts[st[1][1]] = env.expr(st[3:])
        elif st[:3] == [("id", "parsers"), ("op", "."), ("id", "add")]:
            v = env.expr(st[3:])
            parsers.append(v)
        elif st[:3] == [("id", "parsers"), ("op", "."), ("id", "addAll")]:
            parsers.extend(env.expr(st[3:]))
        elif st[0] == ("id", "addExtraOutput"):
            # addExtraOutput(parsers, tok, field): first parser with that token (:640-649)
            args = split_top(st[2:-1], ",")
            tok, out = env.expr(args[1]), env.expr(args[2])
            for p in parsers:
                if p.token == tok:
                    p.add_out(out.typ, out.name, out.casts)
                    break
        else:
            raise SyntaxError("unhandled statement: " + " ".join(str(x[1]) for x in st[:8]))


def fl_original_tokens(src):
    """createFirstAndLastTokenParsers' case labels before the first break (:675-690)"""
    for params, body in src.methods("createFirstAndLastTokenParsers"):
        if any(x == ("id", "switch") for x in body):
            labels = []
            for i, x in enumerate(body):
                if x == ("id", "break"):
                    return labels
                if x == ("id", "case") and body[i + 1][0] == "str":
                    labels.append(body[i + 1][1])
    raise LookupError("createFirstAndLastTokenParsers switch not found")


def extract(root):
    files = {}

    def src(rel):
        s = Src(root, rel)
        files[rel] = s.sha256
        return s

    consts = {}
    base = Env(consts, {}, ())
    casts_constants(src(CASTS), consts, base)
    string_constants(src(TOKENPARSER), consts, base)
    string_constants(src(FIRSTLINE), consts, base)

    apache = src(APACHE)
    env = Env(dict(consts), helper_funcs(apache), set(fl_original_tokens(apache)))
    ap = []
    run_body(apache.method_body("createAllTokenParsers")[1], env, ap)

    nginx = src(NGINX)
    mods = []
    t = nginx.toks
    for i in range(len(t) - 4):
        if t[i:i + 3] == [("id", "modules"), ("op", "."), ("id", "add")] and t[i + 4] == ("id", "new"):
            mods.append(t[i + 5][1])
    ng = []
    for m in mods:
        ms = src(MODULES + m + ".java")
        mc = dict(consts)
        string_constants(ms, mc, Env(mc, {}, ()))
        run_body(ms.method_body("getTokenParsers")[1], Env(mc, helper_funcs(ms), ()), ng)
    return {
        "note": "generated by tests/golden/extract_token_tables.py from the reference's Java sources; do not edit",
        "sources": files,
        "nginx_modules": mods,
        "fl_original_tokens": fl_original_tokens(apache),
        "apache": [p.json() for p in ap],
        "nginx": [p.json() for p in ng],
    }


def main():
    root = sys.argv[1] if len(sys.argv) > 1 else "/root/reference"
    out = sys.argv[2] if len(sys.argv) > 2 else OUT
    tables = extract(root)
    with open(out, "w", encoding="utf-8") as f:
        json.dump(tables, f, indent=1, ensure_ascii=False)
        f.write("\n")
    print("apache %d parsers, nginx %d parsers (%s) -> %s" %
          (len(tables["apache"]), len(tables["nginx"]), ", ".join(tables["nginx_modules"]), out))


if __name__ == "__main__":
    main()
