"""Test corpora built from the synthetic workloads: CRLF / lone-CR line ends
(Hadoop LineRecordReader terminators) and UTF-8 text in the fields.  Shared
by the CPU (emulated) and GPU parity tests."""
import random

# UTF-8 user agents: 2-, 3- and 4-byte chars, none of U+0085 / U+2028 / U+2029
UAS = [
    "Mozilla/5.0 (Linux; Android 13; Pixel 7) AppleWebKit/537.36 (KHTML, wie Gecko) Größe/1.0",
    "Mozilla/5.0 (Windows NT 10.0; Win64; x64) Çà et là – “Navigateur” 2.1",
    "Mozilla/5.0 (iPhone; CPU iPhone OS 17_0 like Mac OS X) 日本語ブラウザ/3.0 Mobile",
    "Mozilla/5.0 (X11; Linux x86_64) ΑΒΓ-Browser/4.2 \U0001F680 rocket",
    "curl/8.0 ünïcödé ñ ø å  nbsp € euro",
    "Bot/1.0 (+https://example.com/bot) 中文 \U0001F600\U0001F4A9",
]
USERS = ["jürgen", "zoë", "李雷", "ōsaka"]


def _fields(line):
    """(prefix up to the referer's opening quote, referer, ua) of a combined line"""
    head, ua = line.rsplit(b' "', 1)
    head, ref = head.rsplit(b' "', 1)
    return head, ref[:-1], ua[:-1]


def utf8_ua_lines(lines, seed):
    """combined lines with a UTF-8 user agent (and sometimes a UTF-8 user):
    every line stays on the device fast path"""
    rng = random.Random(seed)
    out = []
    for l in lines:
        head, ref, _ = _fields(l)
        ua = rng.choice(UAS).encode()
        if rng.random() < 0.2:
            parts = head.split(b" ", 3)
            parts[2] = rng.choice(USERS).encode()
            head = b" ".join(parts)
        out.append(head + b' "' + ref + b'" "' + ua + b'"')
    return out


def utf8_hard_lines(lines, seed):
    """UTF-8 corners: raw UTF-8 in URIs (FALLBACK: URIUtil keeps the bytes and
    the dissector reads them as US-ASCII), U+0085 / U+2028 / U+2029 (not
    matched by '.'), invalid / overlong / surrogate sequences"""
    rng = random.Random(seed)
    bad_seqs = [b"\xc2\x85", b"\xe2\x80\xa8", b"\xe2\x80\xa9", b"\xff", b"\xc0\xaf", b"\xed\xa0\x80",
                b"\xf4\x90\x80\x80", b"\xe0\x80\xaf", b"\xc3", b"\xe6\x97"]
    out = []
    for l in lines:
        head, ref, ua = _fields(l)
        k = rng.randrange(5)
        if k == 0:
            ua = ua[:10] + rng.choice(bad_seqs) + ua[10:]
        elif k == 1:
            ref = ref + "?q=größe&x=日本".encode()
        elif k == 2:
            i = head.index(b'"') + 1
            sp = head.index(b" ", i) + 1
            head = head[:sp] + "/ünï".encode() + head[sp:]
        elif k == 3:
            ua = rng.choice(UAS).encode()
        else:
            ua = ua + rng.choice(bad_seqs[:3])
        out.append(head + b' "' + ref + b'" "' + ua + b'"')
    return out


def crlf_join(lines, seed, lone_cr=0.1):
    """one buffer: "\\r\\n" after most lines, a lone '\\r' after some (a line
    terminator too), '\\n' after the rest; a final line without terminator"""
    rng = random.Random(seed)
    parts = []
    for i, l in enumerate(lines):
        r = rng.random()
        term = b"\r" if r < lone_cr else b"\n" if r < lone_cr + 0.1 else b"\r\n"
        parts.append(l + (term if i + 1 < len(lines) else b""))
    return b"".join(parts)


def split_hadoop(data):
    """Hadoop LineReader.readDefaultLine: '\\n', '\\r' or "\\r\\n" end a line; a
    last line without a terminator counts"""
    out, s, i, n = [], 0, 0, len(data)
    while i < n:
        c = data[i]
        if c == 0x0A or c == 0x0D:
            out.append(data[s:i])
            if c == 0x0D and i + 1 < n and data[i + 1] == 0x0A:
                i += 1
            s = i + 1
        i += 1
    if s < n:
        out.append(data[s:])
    return out
