"""ctypes binding of the CPU oracle (oracle/_build/liboracle.so).

TEST INFRASTRUCTURE ONLY: the oracle is the checker, never the product.
Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg use it.
"""
import ctypes
import json
import os
import subprocess

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
# LP_ORACLE_LIB: another build of the same sources (the ASan/UBSan one, tools/asan_check.sh)
LIB = os.environ.get("LP_ORACLE_LIB") or os.path.join(ROOT, "oracle", "_build", "liboracle.so")

OK, BAD, UNSUPPORTED = 0, 1, 2

_lib = None


def build():
    subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "oracle")], check=True)


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB):
            build()
        L = ctypes.CDLL(LIB)
        L.orc_new.restype = ctypes.c_void_p
        L.orc_new.argtypes = [ctypes.c_char_p, ctypes.POINTER(ctypes.c_char_p), ctypes.c_int,
                              ctypes.c_char_p, ctypes.c_int]
        L.orc_new_remapped.restype = ctypes.c_void_p
        L.orc_new_remapped.argtypes = [ctypes.c_char_p, ctypes.POINTER(ctypes.c_char_p), ctypes.c_int,
                                       ctypes.POINTER(ctypes.c_char_p), ctypes.POINTER(ctypes.c_char_p), ctypes.c_int,
                                       ctypes.c_char_p, ctypes.c_int]
        L.orc_free.argtypes = [ctypes.c_void_p]
        L.orc_parse.restype = ctypes.c_int
        L.orc_parse.argtypes = [ctypes.c_void_p, ctypes.c_char_p, ctypes.c_int, ctypes.c_char_p, ctypes.c_int]
        L.orc_possible_paths.restype = ctypes.c_int
        L.orc_possible_paths.argtypes = [ctypes.c_char_p, ctypes.c_int, ctypes.c_char_p, ctypes.c_int]
        L.orc_format_regex.restype = ctypes.c_int
        L.orc_format_regex.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_char_p, ctypes.c_int]
        L.orc_bench.restype = ctypes.c_double
        L.orc_bench.argtypes = [ctypes.c_char_p, ctypes.POINTER(ctypes.c_char_p), ctypes.c_int,
                                ctypes.c_char_p, ctypes.c_size_t, ctypes.c_int, ctypes.POINTER(ctypes.c_int64)]
        L.orc_resilient_url_decode.restype = ctypes.c_int
        L.orc_resilient_url_decode.argtypes = [ctypes.c_char_p, ctypes.c_int, ctypes.c_char_p, ctypes.c_int]
        L.orc_token_table.restype = ctypes.c_int
        L.orc_token_table.argtypes = [ctypes.c_int, ctypes.c_char_p, ctypes.c_int]
        L.orc_digest_lines.restype = ctypes.c_int64
        L.orc_digest_lines.argtypes = [ctypes.c_char_p, ctypes.POINTER(ctypes.c_char_p), ctypes.c_int, ctypes.c_char_p,
                                       ctypes.c_size_t, ctypes.c_int, ctypes.c_int64, ctypes.c_void_p, ctypes.c_void_p]
        L.orc_digest_lines_w.restype = ctypes.c_int64
        L.orc_digest_lines_w.argtypes = [ctypes.c_char_p, ctypes.POINTER(ctypes.c_char_p), ctypes.c_int,
                                         ctypes.c_char_p, ctypes.c_size_t, ctypes.c_int, ctypes.c_int64,
                                         ctypes.c_int64, ctypes.c_void_p, ctypes.c_void_p]
        L.dg_engine.restype = ctypes.c_int
        L.dg_engine.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64,
                                ctypes.c_int, ctypes.c_void_p]
        _lib = L
    return _lib


def _fields(fields):
    arr = (ctypes.c_char_p * max(1, len(fields)))()
    for i, f in enumerate(fields):
        arr[i] = f.encode()
    return arr


class OracleError(Exception):
    pass


class Oracle:
    """One oracle parser (the reference's Parser is stateful: sticky format)."""

    def __init__(self, logformat, fields, remaps=()):
        """remaps: [(input path, new TYPE)] (Parser.addTypeRemapping)"""
        L = lib()
        err = ctypes.create_string_buffer(512)
        self._fields = _fields(fields)
        self._rm = (_fields([r[0] for r in remaps]), _fields([r[1] for r in remaps]))
        self.h = L.orc_new_remapped(logformat.encode(), self._fields, len(fields), self._rm[0], self._rm[1],
                                    len(remaps), err, 512)
        if not self.h:
            raise OracleError(err.value.decode())
        self.buf = ctypes.create_string_buffer(1 << 20)

    def parse_raw(self, line):
        if isinstance(line, str):
            line = line.encode("utf-8")
        st = lib().orc_parse(self.h, line, len(line), self.buf, len(self.buf))
        if st < 0:
            raise OracleError("output buffer too small")
        return st, (self.buf.value.decode("utf-8") if st == OK else None)

    def parse(self, line):
        st, js = self.parse_raw(line)
        return st, (json.loads(js) if js is not None else None)

    def regex(self, i=0):
        out = ctypes.create_string_buffer(1 << 16)
        n = lib().orc_format_regex(self.h, i, out, len(out))
        return out.value.decode() if n >= 0 else None

    def __del__(self):
        try:
            if self.h:
                lib().orc_free(self.h)
        except Exception:
            pass


def possible_paths(logformat, max_depth=15):
    out = ctypes.create_string_buffer(1 << 20)
    n = lib().orc_possible_paths(logformat.encode(), max_depth, out, len(out))
    if n < 0:
        raise OracleError("possible paths failed")
    return [p for p in out.value.decode().split("\n") if p]


def resilient_url_decode(s):
    b = s.encode("utf-8")
    out = ctypes.create_string_buffer(len(b) * 4 + 16)
    n = lib().orc_resilient_url_decode(b, len(b), out, len(out))
    if n == -2:
        raise ValueError("IllegalArgumentException")
    if n < 0:
        raise OracleError("unsupported")
    return out.raw[:n].decode("utf-8")


def bench(logformat, fields, data, threads):
    out = (ctypes.c_int64 * 4)()
    f = _fields(fields)
    secs = lib().orc_bench(logformat.encode(), f, len(fields), data, len(data), threads, out)
    return secs, list(out)


def token_table(nginx):
    """oracle.c's Apache (False) / NGINX (True) token table, canonical form"""
    out = ctypes.create_string_buffer(1 << 20)
    n = lib().orc_token_table(1 if nginx else 0, out, len(out))
    if n < 0:
        raise OracleError("token table buffer too small")
    return json.loads(out.value.decode("utf-8"))


def digest_lines(logformat, fields, data, threads, max_lines, warmup=0):
    """orc_digest_lines_w: (status u8[n], FNV-1a of each OK line's record u64[n])
    of every '\\n'-terminated line of data, on `threads` threads (several
    LogFormats: each thread's parser warmed up on the `warmup` lines before
    its range, see oracle/digest.c)."""
    import numpy as np
    st = np.zeros(max_lines, dtype=np.uint8)
    h = np.zeros(max_lines, dtype=np.uint64)
    f = _fields(fields)
    n = lib().orc_digest_lines_w(logformat.encode(), f, len(fields), data, len(data), threads, max_lines, warmup,
                                 st.ctypes.data, h.ctypes.data)
    if n < 0:
        raise OracleError("orc_digest_lines failed: %d" % n)
    return st[:n], h[:n]


def digest_engine(record_json_fn, handle, res_ptr, status, threads):
    """dg_engine: the same digest of the engine's records of a host result
    (record_json_fn: the address of the product's lp_result_record_json)."""
    import numpy as np
    h = np.zeros(len(status), dtype=np.uint64)
    st = np.ascontiguousarray(status, dtype=np.uint8)
    rc = lib().dg_engine(record_json_fn, handle, res_ptr, st.ctypes.data, len(st), threads, h.ctypes.data)
    if rc != 0:
        raise OracleError("dg_engine failed: %d" % rc)
    return h
