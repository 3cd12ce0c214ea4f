"""The caller's side of a parse: Parser.store and its setter rules.

Host mirror of parser-core's setter plumbing for the values the engine
delivers (the Parsable.addDissection stream of lp_result_emit):

  * SetterPolicy (core/Parser.java:51-60): ALWAYS / NOT_NULL / NOT_EMPTY;
  * Parser.store (core/Parser.java:760-876): the casts of the target
    (lp_casts = castsOfTargets, or the wildcard / remapped entry) choose which
    of a target's setters run, each receiving Value.getString / getLong /
    getDouble (core/Value.java:48-87); no setter called ->
    FatalErrorDuringCallOfSetterMethod;
  * type remapping (core/Parser.java:636-677, Parsable.java:160-176): a value
    delivered at a remapped name is also delivered under each new type, whose
    casts are STRING_ONLY unless given.  The engine takes care of what the
    new type's dissectors produce (lp_compile_remapped: a remapped query
    parameter dissected as an HTTP.URI runs as a derived URI stage on the
    device); the emissions hold the original delivery only, and this module
    replays the remapped one into the setters.
"""
import enum
import inspect
import math
import re

CAST_STRING, CAST_LONG, CAST_DOUBLE = 1, 2, 4
STRING_ONLY = CAST_STRING
STRING_OR_LONG = CAST_STRING | CAST_LONG
STRING_OR_DOUBLE = CAST_STRING | CAST_DOUBLE
STRING_OR_LONG_OR_DOUBLE = CAST_STRING | CAST_LONG | CAST_DOUBLE
NO_CASTS = 0


class SetterPolicy(enum.Enum):
    ALWAYS = 0     # Normal, empty and null values
    NOT_NULL = 1   # Normal and empty values
    NOT_EMPTY = 2  # Normal values only


class FatalErrorDuringCallOfSetterMethod(Exception):
    pass


_LONG_RE = re.compile(r"[+-]?[0-9]+\Z")
_DEC_RE = re.compile(r"[+-]?(NaN|Infinity|(([0-9]+\.?[0-9]*|\.[0-9]+)([eE][+-]?[0-9]+)?))[fFdD]?\Z")
_HEX_RE = re.compile(r"([+-]?)0[xX]([0-9a-fA-F]+\.?[0-9a-fA-F]*|\.[0-9a-fA-F]+)[pP]([+-]?[0-9]+)[fFdD]?\Z")


def java_parse_long(s):
    """Long.parseLong, None where it throws NumberFormatException"""
    if not _LONG_RE.match(s):
        return None
    v = int(s)
    return v if -(1 << 63) <= v < (1 << 63) else None


def java_parse_double(s):
    """Double.parseDouble (FloatingDecimal.readJavaFormatString: chars <= ' '
    trimmed, optional f/F/d/D suffix, NaN / Infinity, hex floats), None where
    it throws NumberFormatException"""
    t = s.strip("".join(chr(c) for c in range(0x21)))
    m = _DEC_RE.match(t)
    if m:
        body = t.rstrip("fFdD") if not t.endswith("Infinity") and not t.endswith("NaN") else t
        if "NaN" in body:
            return math.nan
        if "Infinity" in body:
            return -math.inf if body.startswith("-") else math.inf
        return float(body)
    m = _HEX_RE.match(t)
    if m:
        sign, mant, exp = m.groups()
        return float.fromhex("%s0x%sp%s" % (sign, mant, exp))
    return None


def java_double_to_string(d):
    """Double.toString: "NaN", "Infinity", plain decimal with at least one
    fraction digit for 1e-3 <= |d| < 1e7, else computerized scientific
    notation ("1.0E7"); shortest round-trip digits.

    The digits are those of JDK 19+ (JDK-4511638, shortest round trip).  The
    reference's pinned JDK 8 (FloatingDecimal.dtoa) prints more digits for
    some values (e.g. 8.41E21 as "8.409999999999999E21").  Parity unpinned:
    no reference test covers it, and no dissector on this path delivers a
    DOUBLE value (only the out-of-scope GeoIP ones do), so getString of a
    Double is reached only through a caller's own setter types."""
    if math.isnan(d):
        return "NaN"
    if math.isinf(d):
        return "Infinity" if d > 0 else "-Infinity"
    if d == 0:
        return "-0.0" if math.copysign(1.0, d) < 0 else "0.0"
    a = abs(d)
    if 1e-3 <= a < 1e7:
        r = repr(d)
        if "e" in r or "E" in r:
            r = format(d, "f")
        return r if "." in r else r + ".0"
    m, e = ("%r" % d).lower().split("e") if "e" in repr(d) else (repr(d), "0")
    digits = m.replace("-", "").replace(".", "").lstrip("0")
    sign = "-" if d < 0 else ""
    exp = int(e) + (len(m.replace("-", "").split(".")[0]) - 1)
    # normalise to one digit before the point
    ip = m.replace("-", "").split(".")[0].lstrip("0")
    if not ip:  # 0.000ddd form
        fr = m.replace("-", "").split(".")[1]
        lead = len(fr) - len(fr.lstrip("0"))
        exp = int(e) - lead - 1
    digits = digits.rstrip("0") or "0"
    return "%s%s.%sE%d" % (sign, digits[0], digits[1:] or "0", exp)


class Value:
    """core/Value.java: one delivered value, filled as a String (or null), a
    Long (int) or a Double (float)"""

    __slots__ = ("filled", "v")

    def __init__(self, v):
        if isinstance(v, bool) or not isinstance(v, (int, float)):
            self.filled = "STRING"
        else:
            self.filled = "LONG" if isinstance(v, int) else "DOUBLE"
        self.v = v

    def get_string(self):
        if self.v is None:
            return None
        if self.filled == "LONG":
            return str(self.v)
        if self.filled == "DOUBLE":
            return java_double_to_string(self.v)
        return self.v

    def get_long(self):
        if self.v is None:
            return None
        if self.filled == "LONG":
            return self.v
        if self.filled == "DOUBLE":
            return int(math.floor(self.v + 0.5))  # Value.java:68: rounding
        return java_parse_long(self.v)

    def get_double(self):
        if self.v is None:
            return None
        if self.filled == "LONG":
            return float(self.v)
        if self.filled == "DOUBLE":
            return self.v
        return java_parse_double(self.v)


class Target:
    """one addParseTarget(method, policy, field) registration.  setter: the
    name of a method of the record (looked up on the record at parse time, as
    the reference resolves the Method on RECORD's class) or any callable; it
    receives (value), or (name, value) when it takes two arguments."""

    def __init__(self, setter, policy, value_class):
        if value_class not in (str, int, float):
            raise ValueError("setter value class must be str (String), int (Long) or float (Double)")
        if not (isinstance(setter, str) or callable(setter)):
            raise ValueError("setter must be a method name or a callable")
        self.setter = setter
        self.policy = policy
        self.value_class = value_class

    def call(self, record, name, v):
        f = getattr(record, self.setter) if isinstance(self.setter, str) else self.setter
        if _arity(f) >= 2:
            f(name, v)
        else:
            f(v)


def _arity(f):
    try:
        return len([p for p in inspect.signature(f).parameters.values()
                    if p.kind in (p.POSITIONAL_ONLY, p.POSITIONAL_OR_KEYWORD)])
    except (TypeError, ValueError):
        return 1


def store(record, key, name, value, targets, casts):
    """Parser.store (core/Parser.java:760-876)"""
    if value is None:
        return
    methods = targets.get(key)
    if not methods:
        return
    casts_to = casts(key)
    if casts_to is None:
        casts_to = casts(name)
        if casts_to is None:
            return
    called = False
    skip = (SetterPolicy.NOT_NULL, SetterPolicy.NOT_EMPTY)
    for t in methods:
        if t.value_class is str:
            if casts_to & CAST_STRING:
                s = value.get_string()
                if s is None:
                    if t.policy in skip:
                        called = True
                        continue
                elif s == "" and t.policy == SetterPolicy.NOT_EMPTY:
                    called = True
                    continue
                t.call(record, name, s)
                called = True
            continue
        if t.value_class is int:
            if casts_to & CAST_LONG:
                v = value.get_long()
                if v is None and t.policy in skip:
                    called = True
                    continue
                t.call(record, name, v)
                called = True
            continue
        if casts_to & CAST_DOUBLE:
            v = value.get_double()
            if v is None and t.policy in skip:
                called = True
                continue
            t.call(record, name, v)
            called = True
    if not called:
        raise FatalErrorDuringCallOfSetterMethod("No setter called for  key = \"%s\"  name = \"%s\"  value = \"%s\""
                                                 % (key, name, value.v))


def cleanup_field_value(field):
    """Parser.cleanupFieldValue (core/Parser.java:681-693): TYPE upper-case, name lower-case"""
    if ":" not in field:
        return field.lower()
    t, n = field.split(":", 1)
    return t.upper() + ":" + n.lower()


def deliver(emissions, record, targets, casts, remaps):
    """Replays Parsable.addDissection (core/Parsable.java:142-193) for one
    line's emissions [(base, type, name, value)] into the setters."""
    for base, typ, name, v in emissions:
        _add(record, base, typ, name, Value(v), targets, casts, remaps, False)
    return record


def _add(record, base, typ, name, value, targets, casts, remaps, recursion):
    if base == "":
        complete, wild = name, typ + ":*"
    else:
        complete = base if name == "" else base + "." + name
        wild = typ + ":" + base + ".*"
    needed = typ + ":" + complete
    if not recursion:
        for nt in sorted(remaps.get(complete, ())):
            if nt == typ:
                raise ValueError("[Type Remapping] Trying to map to the same type (mapping definition bug!):  base=%s "
                                 "type=%s name=%s" % (base, typ, name))
            _add(record, base, nt, name, value, targets, casts, remaps, True)
    if needed in targets:
        store(record, needed, needed, value, targets, casts)
    if wild in targets:
        store(record, wild, needed, value, targets, casts)
