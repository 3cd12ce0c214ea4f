"""strftime test corpus (StrfTimeStampDissector, every conversion the
reference converts): values printed from random date-times the way the
reference's DateTimeFormatter prints them (en_US text, US week-based year
for %G / %g, ISO week-of-year for %V / %W, Apache's msec_frac), some of them
mutated (wrong day names, conflicting hours, out-of-range fields, stray
bytes), inside a small LogFormat.  Shared by the CPU (emulated) and GPU
parity tests; the oracle decides every line."""
import datetime
import random

MON = ["January", "February", "March", "April", "May", "June", "July", "August", "September", "October",
       "November", "December"]
DOW = ["Monday", "Tuesday", "Wednesday", "Thursday", "Friday", "Saturday", "Sunday"]

# patterns: the reference's own MultiFields pattern, and shorter realistic ones
PATTERNS = [
    "%D %F %R %T %r %a %A %b %B %d %G %h %H %I %j %k %l %m %M %p %s %S %u %Y %z",
    "%a, %d %b %Y %T %z",
    "%A %B %e %Y %l:%M:%S %p %z",
    "%s",
    "%s.msec_frac %z",
    "%D %r",
    "%Y-%j %H:%M",
    "%G %V %u %Y %m %d %T",
    "%y%m%d %k:%M:%S",
    "%d/%b/%Y %I:%M %P",
    "%F %R:%S.usec_frac %Z",
    "%a %b %e %H:%M:%S %Y",
    "%W %F %T",
]


def _week_fields(d, sow, mind):
    """(weekOfYear, weekBasedYear) of WeekFields(sow 1=Mon..7=Sun, minimal days)"""
    def offset(day, ldow):
        ws = (day - ldow) % 7
        return 7 - ws if ws + 1 > mind else -ws
    ldow = (d.isoweekday() - sow) % 7 + 1
    doy = d.timetuple().tm_yday
    off = offset(doy, ldow)
    week = (7 + off + doy - 1) // 7
    ylen = 366 if (d.year % 4 == 0 and (d.year % 100 != 0 or d.year % 400 == 0)) else 365
    wby = d.year - 1 if week == 0 else (d.year + 1 if week >= (7 + off + ylen + mind - 1) // 7 else d.year)
    return week, wby


def render(pattern, dt, off_min):
    """the value java.time prints for dt (local, offset minutes off_min)"""
    out, i = [], 0
    woy, _ = _week_fields(dt, 1, 4)
    _, wby = _week_fields(dt, 7, 1)
    epoch = int((dt - datetime.timedelta(minutes=off_min) - datetime.datetime(1970, 1, 1)).total_seconds())
    h12 = dt.hour % 12 or 12
    sign = "-" if off_min < 0 else "+"
    conv = {
        "a": DOW[dt.weekday()][:3], "A": DOW[dt.weekday()], "b": MON[dt.month - 1][:3], "h": MON[dt.month - 1][:3],
        "B": MON[dt.month - 1], "d": "%02d" % dt.day, "D": "%02d/%02d/%02d" % (dt.month, dt.day, dt.year % 100),
        "e": "%2d" % dt.day, "F": "%04d-%02d-%02d" % (dt.year, dt.month, dt.day), "G": "%04d" % wby,
        "g": "%02d" % (wby % 100), "H": "%02d" % dt.hour, "I": "%02d" % h12, "j": "%03d" % dt.timetuple().tm_yday,
        "k": "%2d" % dt.hour, "l": "%2d" % h12, "m": "%02d" % dt.month, "M": "%02d" % dt.minute,
        "p": "AM" if dt.hour < 12 else "PM", "P": "am" if dt.hour < 12 else "pm",
        "r": "%02d:%02d:%02d %s" % (h12, dt.minute, dt.second, "AM" if dt.hour < 12 else "PM"),
        "R": "%02d:%02d" % (dt.hour, dt.minute), "s": str(epoch), "S": "%02d" % dt.second,
        "T": "%02d:%02d:%02d" % (dt.hour, dt.minute, dt.second), "u": str(dt.isoweekday()), "V": str(woy),
        "W": "%02d" % woy, "y": "%02d" % (dt.year % 100), "Y": "%04d" % dt.year,
        "z": "%s%02d%02d" % (sign, abs(off_min) // 60, abs(off_min) % 60), "Z": "UTC",
    }
    while i < len(pattern):
        if pattern.startswith("msec_frac", i):
            out.append("%03d" % (dt.microsecond // 1000)); i += 9
        elif pattern.startswith("usec_frac", i):
            out.append("%06d" % dt.microsecond); i += 9
        elif pattern[i] == "%" and i + 1 < len(pattern):
            out.append(conv[pattern[i + 1]]); i += 2
        else:
            out.append(pattern[i]); i += 1
    return "".join(out)


def mutate(rng, v):
    r = rng.random()
    b = list(v)
    if r < 0.25 and b:  # a different digit
        k = rng.randrange(len(b))
        if b[k].isdigit():
            b[k] = str((int(b[k]) + rng.randint(1, 9)) % 10)
    elif r < 0.4:  # another day / month name
        for names in (DOW, MON):
            for n in names:
                if n[:3] in v:
                    return v.replace(n[:3], rng.choice(names)[:3], 1)
    elif r < 0.55 and b:  # a byte dropped
        del b[rng.randrange(len(b))]
    elif r < 0.7:  # case changed
        return v.swapcase()
    elif r < 0.8:  # AM <-> PM
        return v.replace("AM", "PM") if "AM" in v else v.replace("PM", "AM")
    elif r < 0.9 and b:  # a space or stray byte inserted
        b.insert(rng.randrange(len(b) + 1), rng.choice([" ", "0", "x", "+"]))
    else:  # a non-ASCII letter java folds to ASCII (U+017F long s)
        return v.replace("s", "ſ", 1)
    return "".join(b)


def corpus(seed, per_pattern=150):
    """[(logformat, [line bytes])]: each pattern inside '%h [%{...}t] "%r"'"""
    rng = random.Random(seed)
    out = []
    for pat in PATTERNS:
        lines = []
        for k in range(per_pattern):
            dt = datetime.datetime(1971, 1, 1) + datetime.timedelta(seconds=rng.randrange(0, 60 * 365 * 86400),
                                                                    microseconds=rng.randrange(1000000))
            if k % 7 == 0:  # around new year (week-based years) and midnight / noon
                dt = datetime.datetime(rng.randint(1990, 2030), rng.choice([1, 12]), rng.choice([1, 2, 3, 29, 30, 31]),
                                       rng.choice([0, 11, 12, 23]), rng.randrange(60), rng.randrange(60))
            off = rng.choice([0, 60, -300, 330, 570, -600])
            v = render(pat, dt, 0 if "%z" not in pat else off)
            if k % 3 == 1:
                v = mutate(rng, v)
            lines.append(('10.1.2.%d [%s] "GET /x HTTP/1.1"' % (k % 250, v)).encode("utf-8"))
        out.append(('%h [%{' + pat + '}t] "%r"', lines))
    return out


FIELDS = ["TIME.EPOCH:request.receive.time.epoch", "TIME.DATE:request.receive.time.date",
          "TIME.TIME:request.receive.time.time", "TIME.DATE:request.receive.time.date_utc",
          "TIME.TIME:request.receive.time.time_utc", "TIME.WEEK:request.receive.time.weekofweekyear",
          "TIME.YEAR:request.receive.time.weekyear", "TIME.MILLISECOND:request.receive.time.millisecond",
          "TIME.NANOSECOND:request.receive.time.nanosecond", "IP:connection.client.host"]
