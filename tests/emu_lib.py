"""TEST-ONLY ctypes binding of tests/emu (CPU emulation of the device per-line
code, compiled from logparser_amd/csrc/lp_device.h with g++).  Lets the CPU
test suite diff the device logic against the oracle; never used by the
product or the benchmark."""
import ctypes
import json
import os
import subprocess

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(ROOT, "tests", "emu", "_build", "libemu.so")
# ASan/UBSan build of the same sources (tools/asan_check.sh sets LP_EMU_ASAN=1)
ASAN = os.environ.get("LP_EMU_ASAN") == "1"
SAN_FLAGS = ["-fsanitize=address,undefined", "-fno-sanitize-recover=undefined", "-fno-omit-frame-pointer"]
if ASAN:
    LIB = os.path.join(ROOT, "tests", "emu", "_build", "libemu_asan.so")
SRCS = [os.path.join(ROOT, "tests", "emu", "emu.cpp"), os.path.join(ROOT, "logparser_amd", "csrc", "plan.cpp")]
HDRS = [os.path.join(ROOT, "logparser_amd", "csrc", h) for h in ("lp_device.h", "lp_program.h", "plan.h")]

_lib = None


def build(force=False):
    newest = max(os.path.getmtime(p) for p in SRCS + HDRS)
    if not force and os.path.exists(LIB) and os.path.getmtime(LIB) >= newest:
        return
    os.makedirs(os.path.dirname(LIB), exist_ok=True)
    flags = ["-O1"] + SAN_FLAGS if ASAN else ["-O2"]
    # built under a private name and renamed into place: parallel test
    # workers never load a half-written library
    tmp = "%s.%d.tmp" % (LIB, os.getpid())
    subprocess.run(["g++", "-std=c++17", "-g", "-fPIC", "-shared", "-o", tmp] + flags + SRCS, check=True)
    os.replace(tmp, LIB)


def lib():
    global _lib
    if _lib is None:
        build()
        L = ctypes.CDLL(LIB)
        L.emu_new.restype = ctypes.c_void_p
        L.emu_new.argtypes = [ctypes.c_char_p, ctypes.POINTER(ctypes.c_char_p), ctypes.c_int,
                              ctypes.POINTER(ctypes.c_int), ctypes.c_char_p, ctypes.c_int]
        L.emu_new_remapped.restype = ctypes.c_void_p
        L.emu_new_remapped.argtypes = [ctypes.c_char_p, ctypes.POINTER(ctypes.c_char_p), ctypes.c_int,
                                       ctypes.POINTER(ctypes.c_char_p), ctypes.POINTER(ctypes.c_char_p), ctypes.c_int,
                                       ctypes.POINTER(ctypes.c_int), ctypes.c_char_p, ctypes.c_int]
        L.emu_free.argtypes = [ctypes.c_void_p]
        L.emu_parse.restype = ctypes.c_int
        L.emu_parse.argtypes = [ctypes.c_void_p, ctypes.c_char_p, ctypes.c_int, ctypes.c_char_p, ctypes.c_int]
        L.emu_parse_in.restype = ctypes.c_int
        L.emu_parse_in.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64, ctypes.c_int, ctypes.c_char_p,
                                   ctypes.c_int]
        L.emu_describe.argtypes = [ctypes.c_void_p, ctypes.c_char_p, ctypes.c_int]
        L.emu_set_masks.argtypes = [ctypes.c_int]
        L.emu_casts.restype = ctypes.c_int
        L.emu_casts.argtypes = [ctypes.c_void_p, ctypes.c_char_p]
        L.emu_possible_paths.argtypes = [ctypes.c_char_p, ctypes.c_int, ctypes.c_char_p, ctypes.c_int]
        L.emu_token_table.restype = ctypes.c_int
        L.emu_token_table.argtypes = [ctypes.c_int, ctypes.c_char_p, ctypes.c_int]
        L.emu_uplist.argtypes = [ctypes.c_char_p, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                 ctypes.POINTER(ctypes.c_int)]
        L.emu_uplist_items.restype = ctypes.c_int
        L.emu_uplist_items.argtypes = [ctypes.c_char_p, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                       ctypes.POINTER(ctypes.c_int64)]
        L.emu_strf.restype = ctypes.c_int
        L.emu_strf.argtypes = [ctypes.c_void_p, ctypes.c_char_p, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                               ctypes.POINTER(ctypes.c_int64)]
        _lib = L
    return _lib


def _cstrs(xs):
    arr = (ctypes.c_char_p * max(1, len(xs)))()
    for i, x in enumerate(xs):
        arr[i] = x.encode()
    return arr


class Emu:
    def __init__(self, logformat, fields, remaps=()):
        """remaps: [(input path, new TYPE)] (Parser.addTypeRemapping)"""
        arr = _cstrs(fields)
        self._arr = arr
        self._rm = (_cstrs([r[0] for r in remaps]), _cstrs([r[1] for r in remaps]))
        st = ctypes.c_int(0)
        err = ctypes.create_string_buffer(512)
        self.h = lib().emu_new_remapped(logformat.encode(), arr, len(fields), self._rm[0], self._rm[1], len(remaps),
                                        ctypes.byref(st), err, 512)
        self.status = st.value
        self.err = err.value.decode()
        if not self.h:
            raise RuntimeError("emu compile failed %d: %s" % (self.status, self.err))
        self.buf = ctypes.create_string_buffer(1 << 20)

    def parse(self, line):
        if isinstance(line, str):
            line = line.encode("utf-8")
        st = lib().emu_parse(self.h, line, len(line), self.buf, len(self.buf))
        return st, (json.loads(self.buf.value.decode("utf-8")) if st == 0 else None)

    def parse_raw(self, line):
        if isinstance(line, str):
            line = line.encode("utf-8")
        st = lib().emu_parse(self.h, line, len(line), self.buf, len(self.buf))
        return st, (self.buf.value.decode("utf-8") if st in (0, 3) else None)

    def parse_batch_raw(self, data):
        """Every '\\n'-terminated line of data, each parsed in place inside the
        whole buffer (neighbouring bytes around it, as in the kernel's LDS
        window).  Returns [(status, json or None)]."""
        n = len(data)
        buf = ctypes.create_string_buffer(data + b"\0" * 16, n + 16)
        assert ctypes.addressof(buf) % 4 == 0
        out, start = [], 0
        while start < n:
            end = data.find(b"\n", start)
            if end < 0:
                end = n
            st = lib().emu_parse_in(self.h, ctypes.addressof(buf), start, end - start, self.buf, len(self.buf))
            out.append((st, self.buf.value.decode("utf-8") if st in (0, 3) else None))
            start = end + 1
        return out

    def strf(self, value, off, use_fixed):
        """parse_strf_time of the first time stage on value (bytes) at byte
        offset off of an aligned buffer, with the fixed-layout plan or the
        general loop only: (plan fields, (status, epoch_ms, local, utc, nanos))"""
        out = (ctypes.c_int64 * 5)()
        n = lib().emu_strf(self.h, value, len(value), off, 1 if use_fixed else 0, out)
        return n, tuple(out)

    def casts(self, target):
        c = lib().emu_casts(self.h, target.encode())
        return None if c < 0 else c

    def describe(self):
        b = ctypes.create_string_buffer(1 << 16)
        lib().emu_describe(self.h, b, len(b))
        return b.value.decode()

    def __del__(self):
        try:
            lib().emu_free(self.h)
        except Exception:
            pass


def uplist(line, p, off, dec):
    """(uplist_at, uplist_at_r) of the line (bytes) at p"""
    out = (ctypes.c_int * 2)()
    lib().emu_uplist(line, len(line), p, off, 1 if dec else 0, out)
    return out[0], out[1]


def uplist_items(tok, off, dec):
    """UpstreamListDissector split of the token (bytes) by uplist_items and
    uplist_items_r: ((count, items), (count or -2, items)), an item being
    (va, vb, ra, rb, value ms, redirected ms)"""
    out = (ctypes.c_int64 * (2 + 2 * 16 * 8))()
    lib().emu_uplist_items(tok, len(tok), off, 1 if dec else 0, out)
    res = []
    for v in range(2):
        n = out[v]
        base = 2 + 16 * 8 * v
        items = [tuple(out[base + 8 * k + j] for j in range(6)) for k in range(max(0, min(n, 16)))]
        res.append((n, items))
    return tuple(res)


def possible_paths(logformat, depth=15):
    b = ctypes.create_string_buffer(1 << 20)
    lib().emu_possible_paths(logformat.encode(), depth, b, len(b))
    return [p for p in b.value.decode().split("\n") if p]


def token_table(nginx):
    """plan.cpp's Apache (False) / NGINX (True) token table, canonical form"""
    n = lib().emu_token_table(1 if nginx else 0, None, 0)
    b = ctypes.create_string_buffer(n + 1)
    lib().emu_token_table(1 if nginx else 0, b, len(b))
    return json.loads(b.value.decode("utf-8"))
