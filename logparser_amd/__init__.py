"""logparser_amd -- MI355X-native batch engine for logparser's per-line hot path.

Host-side mirror of the reference's parser surface for this path
(nl.basjes.parse.httpdlog.HttpdLoglineParser / nl.basjes.parse.core.Parser,
reference: httpdlog/httpdlog-parser/src/main/java/nl/basjes/parse/httpdlog/
HttpdLoglineParser.java:44-126 and parser-core/src/main/java/nl/basjes/parse/core/
Parser.java:496-756, 904-1012) over the C ABI in include/logparser_amd.h.

    parser = HttpdLoglineParser("combined", ["TIME.EPOCH:request.receive.time.epoch", ...])
    batch  = parser.parse_batch(raw_bytes_or_cuda_uint8_tensor)   # all lines on the GPU
    batch.status            # per line: OK / BAD (DissectionFailure) / FALLBACK
    batch.record(i)         # {"TYPE:path": [values]} as the reference setters receive them
    parser.parse(line)      # Parser.parse(line) for one line (raises DissectionFailure)

The engine runs only on the GPU: there is no CPU implementation behind this
module, and every call fails loudly when the HIP library or a device is
missing.  FALLBACK lines are the lines the device could not prove it handles
exactly; a deployment hands them to the reference Java dissector.
"""
import ctypes
import json
import os

import numpy as np

from .setters import (CAST_DOUBLE, CAST_LONG, CAST_STRING, NO_CASTS, STRING_ONLY, STRING_OR_DOUBLE,  # noqa: F401
                      STRING_OR_LONG, STRING_OR_LONG_OR_DOUBLE, FatalErrorDuringCallOfSetterMethod, SetterPolicy,
                      Target, cleanup_field_value, deliver)

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("LOGPARSER_AMD_LIB") or os.path.join(_HERE, "_lib", "liblogparser_amd.so")

LP_OK, LP_E_INVALID, LP_E_MISSING, LP_E_UNSUPPORTED, LP_E_DEVICE, LP_E_NOMEM, LP_E_STATE = 0, -1, -2, -3, -4, -5, -6
LINE_OK, LINE_BAD, LINE_FALLBACK = 0, 1, 2
BUF_HOST, BUF_DEVICE = 0, 1
OPT_FORCE_DIRECT, OPT_MAX_RETRIES, OPT_ARENA_BYTES, OPT_CHUNK_LINES, OPT_CHUNK_WAIT, OPT_ONE_PASS = 1, 2, 3, 4, 5, 6
ARENA_SHARDS = 64


class LpColumn(ctypes.Structure):
    """lp_column (include/logparser_amd.h)"""
    _fields_ = [("name", ctypes.c_char * 16), ("index", ctypes.c_int32), ("elem_size", ctypes.c_int32),
                ("offset", ctypes.c_uint64)]


EMIT_FN = ctypes.CFUNCTYPE(None, ctypes.c_void_p, ctypes.c_char_p, ctypes.c_char_p, ctypes.c_char_p, ctypes.c_int,
                           ctypes.POINTER(ctypes.c_uint8), ctypes.c_uint32, ctypes.c_int64)
VALUE_STRING, VALUE_NULL, VALUE_LONG = 0, 1, 2


class LpTableCol(ctypes.Structure):
    _fields_ = [("path", ctypes.c_char_p), ("kind", ctypes.c_int32), ("valid", ctypes.c_void_p),
                ("i64", ctypes.c_void_p), ("f64", ctypes.c_void_p), ("chars", ctypes.c_void_p),
                ("chars_cap", ctypes.c_uint64), ("chars_len", ctypes.c_uint64)]


class LpResult(ctypes.Structure):
    """lp_result (include/logparser_amd.h): the SoA results of one batch"""
    _fields_ = [("n_lines", ctypes.c_int64), ("first_line", ctypes.c_int64), ("input_bytes", ctypes.c_uint64),
                ("input", ctypes.c_void_p),
                ("line_off", ctypes.c_void_p), ("columns", ctypes.c_void_p), ("columns_bytes", ctypes.c_uint64),
                ("arena", ctypes.c_void_p), ("arena_bytes", ctypes.c_uint64), ("shard_cap", ctypes.c_uint64),
                ("shard_off", ctypes.c_uint64 * ARENA_SHARDS), ("n_columns", ctypes.c_int32),
                ("on_host", ctypes.c_int32), ("column", ctypes.POINTER(LpColumn))]


class DissectionFailure(Exception):
    """nl.basjes.parse.core.exceptions.DissectionFailure"""


class FallbackRequired(Exception):
    """The device could not prove the line; hand it to the reference parser."""


class MissingDissectorsException(Exception):
    """nl.basjes.parse.core.exceptions.MissingDissectorsException"""


class InvalidDissectorException(Exception):
    """nl.basjes.parse.core.exceptions.InvalidDissectorException"""


class EngineUnavailable(RuntimeError):
    """The HIP library or a GPU is missing."""


_lib = None


def lib():
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise EngineUnavailable("logparser_amd: %s not built (run __graft_entry__.build())" % LIB_PATH)
    # One HIP runtime per process: torch ships its own libamdhip64.so.7.  If it
    # is loaded first, the engine binds to it (same SONAME) and device pointers
    # and streams are shared; loaded the other way round, two runtimes fight
    # over the device and torch sees no GPU.
    try:
        import torch  # noqa: F401
    except ImportError:
        pass
    L = ctypes.CDLL(LIB_PATH)
    c_char_pp = ctypes.POINTER(ctypes.c_char_p)
    L.lp_compile.restype = ctypes.c_void_p
    L.lp_compile.argtypes = [ctypes.c_char_p, c_char_pp, ctypes.c_int, ctypes.c_int, ctypes.POINTER(ctypes.c_int),
                             ctypes.c_char_p, ctypes.c_size_t]
    L.lp_free.argtypes = [ctypes.c_void_p]
    L.lp_possible_paths.restype = ctypes.c_int64
    L.lp_possible_paths.argtypes = [ctypes.c_char_p, ctypes.c_int, ctypes.c_char_p, ctypes.c_size_t]
    L.lp_compile_remapped.restype = ctypes.c_void_p
    L.lp_compile_remapped.argtypes = [ctypes.c_char_p, c_char_pp, ctypes.c_int, ctypes.POINTER(LpRemap), ctypes.c_int,
                                      ctypes.c_int, ctypes.POINTER(ctypes.c_int), ctypes.c_char_p, ctypes.c_size_t]
    L.lp_possible_paths_remapped.restype = ctypes.c_int64
    L.lp_possible_paths_remapped.argtypes = [ctypes.c_char_p, ctypes.c_int, ctypes.POINTER(LpRemap), ctypes.c_int,
                                             ctypes.c_char_p, ctypes.c_size_t]
    L.lp_parse_batch.restype = ctypes.c_int
    L.lp_parse_batch.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64, ctypes.c_int, ctypes.c_void_p]
    L.lp_parse_batch_at.restype = ctypes.c_int
    L.lp_parse_batch_at.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64, ctypes.c_int64, ctypes.c_int,
                                    ctypes.c_void_p]
    L.lp_sync.argtypes = [ctypes.c_void_p]
    L.lp_num_lines.restype = ctypes.c_int64
    L.lp_num_lines.argtypes = [ctypes.c_void_p]
    L.lp_line_status.argtypes = [ctypes.c_void_p, ctypes.c_int64, ctypes.c_int64, ctypes.c_void_p]
    L.lp_line_offset.restype = ctypes.c_int64
    L.lp_line_offset.argtypes = [ctypes.c_void_p, ctypes.c_int64]
    L.lp_line_record_json.restype = ctypes.c_int64
    L.lp_line_record_json.argtypes = [ctypes.c_void_p, ctypes.c_int64, ctypes.c_char_p, ctypes.c_size_t]
    L.lp_counters.argtypes = [ctypes.c_void_p, ctypes.POINTER(ctypes.c_uint64), ctypes.c_int]
    L.lp_last_timing.argtypes = [ctypes.c_void_p, ctypes.POINTER(ctypes.c_float), ctypes.c_int]
    L.lp_histograms.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int]
    L.lp_last_bytes.argtypes = [ctypes.c_void_p, ctypes.POINTER(ctypes.c_uint64), ctypes.c_int]
    L.lp_set_option.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int64]
    L.lp_reserve.argtypes = [ctypes.c_void_p, ctypes.c_int64, ctypes.c_uint64]
    L.lp_result_view.argtypes = [ctypes.c_void_p, ctypes.POINTER(LpResult)]
    L.lp_result_copy.restype = ctypes.c_int64
    L.lp_result_copy.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64, ctypes.c_int,
                                 ctypes.POINTER(LpResult)]
    L.lp_result_record_json.restype = ctypes.c_int64
    L.lp_result_record_json.argtypes = [ctypes.c_void_p, ctypes.POINTER(LpResult), ctypes.c_int64, ctypes.c_char_p,
                                        ctypes.c_size_t]
    L.lp_result_emit.argtypes = [ctypes.c_void_p, ctypes.POINTER(LpResult), ctypes.c_int64, EMIT_FN, ctypes.c_void_p]
    L.lp_result_table.restype = ctypes.c_int
    L.lp_result_table.argtypes = [ctypes.c_void_p, ctypes.POINTER(LpResult), ctypes.c_int64, ctypes.c_int64,
                                  ctypes.POINTER(LpTableCol), ctypes.c_int, ctypes.c_int]
    L.lp_casts.restype = ctypes.c_int
    L.lp_casts.argtypes = [ctypes.c_void_p, ctypes.c_char_p]
    L.lp_describe.restype = ctypes.c_int64
    L.lp_describe.argtypes = [ctypes.c_void_p, ctypes.c_char_p, ctypes.c_size_t]
    L.lp_synth_combined.restype = ctypes.c_int64
    L.lp_synth_combined.argtypes = [ctypes.c_uint64, ctypes.c_int64, ctypes.c_int64, ctypes.c_void_p, ctypes.c_size_t,
                                    ctypes.POINTER(ctypes.c_int64)]
    L.lp_synth.restype = ctypes.c_int64
    L.lp_synth.argtypes = [ctypes.c_int, ctypes.c_uint64, ctypes.c_int64, ctypes.c_int64, ctypes.c_void_p,
                           ctypes.c_size_t, ctypes.POINTER(ctypes.c_int64)]
    _lib = L
    return L


class LpRemap(ctypes.Structure):
    """lp_remap: Parser.addTypeRemapping(input, type, casts)"""
    _fields_ = [("input", ctypes.c_char_p), ("type", ctypes.c_char_p), ("casts", ctypes.c_int32)]


def _remap_array(remaps):
    """[(input, TYPE, casts)] -> (lp_remap array, count)"""
    arr = (LpRemap * max(1, len(remaps)))()
    for i, (n, t, c) in enumerate(remaps):
        arr[i] = LpRemap(n.encode(), t.encode(), c)
    return arr, len(remaps)


def get_possible_paths(logformat, max_depth=15, remaps=()):
    """Parser.getPossiblePaths(maxDepth) for a HttpdLoglineParser on logformat
    (remaps: [(input, TYPE, casts)], its type remappings)."""
    cap = 1 << 20
    out = ctypes.create_string_buffer(cap)
    arr, n_rm = _remap_array(list(remaps))
    n = lib().lp_possible_paths_remapped(logformat.encode(), max_depth, arr, n_rm, out, cap)
    if n < 0:
        raise InvalidDissectorException("possible paths overflow")
    return [p for p in out.value.decode().split("\n") if p]


def synth_combined(seed, first_line, n_lines):
    """Deterministic synthetic 'combined' lines (BASELINE config 2 shape) as bytes."""
    cap = n_lines * 700 + 1024
    buf = ctypes.create_string_buffer(cap)
    got = ctypes.c_int64(0)
    nb = lib().lp_synth_combined(seed, first_line, n_lines, buf, cap, ctypes.byref(got))
    return buf.raw[:nb]


SYNTH_COMBINED, SYNTH_STRFTIME, SYNTH_NGINX, SYNTH_MIXED = 2, 3, 4, 5

# the LogFormat of each synthetic workload (BASELINE.json configs 2-5)
SYNTH_FORMATS = {
    SYNTH_COMBINED: "combined",
    SYNTH_STRFTIME: '%h %l %u [%{%d/%b/%Y %T}t.%{msec_frac}t] "%r" %>s %b "%{Referer}i" "%{User-Agent}i" %I %O',
    SYNTH_NGINX: '$remote_addr - $remote_user [$time_local] "$request" $status $body_bytes_sent "$http_referer" '
                 '"$http_user_agent" "$http_x_forwarded_for" $request_time $upstream_response_time $pipe',
}
# config 5: the three formats of the mixed corpus, one LogFormat per line, in
# HttpdLogFormatDissector's list order (hp/HttpdLogFormatDissector.java:110-125)
SYNTH_FORMATS[SYNTH_MIXED] = "\n".join((SYNTH_FORMATS[SYNTH_COMBINED], SYNTH_FORMATS[SYNTH_NGINX], "common"))


def synth(workload, seed, first_line, n_lines):
    """Deterministic synthetic lines of a BASELINE.json workload (SYNTH_*) as bytes."""
    cap = n_lines * 800 + 1024
    buf = ctypes.create_string_buffer(cap)
    got = ctypes.c_int64(0)
    nb = lib().lp_synth(workload, seed, first_line, n_lines, buf, cap, ctypes.byref(got))
    if nb < 0:
        raise ValueError("unknown synthetic workload %r" % workload)
    return buf.raw[:nb]


class BatchResult:
    """Results of one parse_batch call (valid until the parser's next batch)."""

    def __init__(self, parser):
        self._p = parser
        L = lib()
        rc = L.lp_sync(parser._h)
        if rc != LP_OK:
            raise EngineUnavailable("lp_sync failed: %d" % rc)
        self.n_lines = L.lp_num_lines(parser._h)
        st = np.zeros(max(1, self.n_lines), dtype=np.uint8)
        if self.n_lines:
            rc = L.lp_line_status(parser._h, 0, self.n_lines, st.ctypes.data)
            if rc != LP_OK:
                raise EngineUnavailable("lp_line_status failed: %d" % rc)
        self.status = st[: self.n_lines]
        c = (ctypes.c_uint64 * 9)()
        L.lp_counters(parser._h, c, 9)
        self.counters = {"lines": c[0], "ok": c[1], "bad": c[2], "fallback": c[3]}
        self.diag = {"overflow_waves": c[4], "retries": c[5], "arena_ovf": c[6], "uri_overflow_waves": c[7],
                     "deferred_chunks": c[8]}
        t = (ctypes.c_float * 3)()
        L.lp_last_timing(parser._h, t, 3)
        self.timing_ms = {"total": t[0], "index": t[1], "parse": t[2]}
        b = (ctypes.c_uint64 * 2)()
        L.lp_last_bytes(parser._h, b, 2)
        self.bytes_in, self.bytes_out = b[0], b[1]

    def record(self, i):
        """Values the reference Parser would deliver for line i (status OK)."""
        return json.loads(self.record_json(i))

    def record_json(self, i):
        cap = 1 << 16
        while True:
            out = ctypes.create_string_buffer(cap)
            n = lib().lp_line_record_json(self._p._h, i, out, cap)
            if n >= 0:
                return out.value.decode("utf-8")
            if n <= -100:
                cap = int(-n - 100) + 16
                continue
            if n == LP_E_STATE:
                raise ValueError("line %d has status %d" % (i, self.status[i]))
            raise EngineUnavailable("lp_line_record_json failed: %d" % n)

    def line_offset(self, i):
        return lib().lp_line_offset(self._p._h, i)

    def histograms(self):
        """lp_histograms into host memory: a dict view of the run counters"""
        return decode_histograms(self._p.histograms())

    def copy_to_host(self, with_input=True, buf=None):
        """lp_result_copy: every result of the batch in one host buffer (a
        numpy uint8 array, or buf when given and large enough); returns
        (buffer, LpResult)."""
        L = lib()
        need = -L.lp_result_copy(self._p._h, None, 0, 1 if with_input else 0, None)
        if need <= 0:
            raise EngineUnavailable("lp_result_copy failed: %d" % need)
        if buf is None or buf.nbytes < need:
            buf = np.empty(need, dtype=np.uint8)
        res = LpResult()
        rc = L.lp_result_copy(self._p._h, buf.ctypes.data, buf.nbytes, 1 if with_input else 0, ctypes.byref(res))
        if rc < 0:
            raise EngineUnavailable("lp_result_copy failed: %d" % rc)
        return buf, res

    def columns(self, res):
        """{(name, index): numpy view} of the columns of a host copy."""
        dt = {1: np.uint8, 2: np.uint16, 4: np.uint32, 8: np.uint64}
        out = {}
        for k in range(res.n_columns):
            c = res.column[k]
            arr = np.ctypeslib.as_array((ctypes.c_uint8 * (c.elem_size * res.n_lines)).from_address(res.columns + c.offset))
            out[(c.name.decode(), c.index)] = arr.view(dt[c.elem_size])
        return out

    def emissions_from(self, res, i):
        """lp_result_emit: the Parsable.addDissection(base, type, name, value)
        calls delivering line i's values, from a host copy with the input;
        value = str | None | int."""
        out = []

        def cb(_ctx, base, typ, name, kind, p, n, l):
            v = None if kind == VALUE_NULL else l if kind == VALUE_LONG else ctypes.string_at(p, n).decode("utf-8")
            out.append((base.decode(), typ.decode(), name.decode(), v))

        fn = EMIT_FN(cb)
        rc = lib().lp_result_emit(self._p._h, ctypes.byref(res), i, fn, None)
        if rc < 0:
            raise ValueError("lp_result_emit(%d) failed: %d" % (i, rc))
        return out

    def table_from(self, res, columns, first=0, count=None, threads=16, decode=True):
        """lp_result_table: typed columns of rows [first, first+count) from a
        host copy.  columns: [(path, str | int | float)].  Returns {path:
        (values, valid)}: values a list of str / None for STRING columns
        (decode=False: the Arrow pair (offsets, chars bytes) as numpy arrays),
        a numpy int64 / float64 array for BIGINT / DOUBLE ones."""
        count = self.n_lines - first if count is None else count
        kinds = {str: CAST_STRING, int: CAST_LONG, float: CAST_DOUBLE}
        cols = (LpTableCol * len(columns))()
        keep = []
        for k, (path, typ) in enumerate(columns):
            c = cols[k]
            c.path = path.encode()
            c.kind = kinds[typ]
            valid = np.zeros(max(1, count), dtype=np.uint8)
            i64 = np.zeros(count + 1, dtype=np.int64)
            f64 = np.zeros(max(1, count), dtype=np.float64)
            c.valid, c.i64, c.f64 = valid.ctypes.data, i64.ctypes.data, f64.ctypes.data
            keep.append((valid, i64, f64))
        L = lib()
        rc = L.lp_result_table(self._p._h, ctypes.byref(res), first, count, cols, len(columns), threads)
        if rc == LP_E_NOMEM:
            for k in range(len(columns)):
                if cols[k].kind == CAST_STRING:
                    buf = np.zeros(max(1, cols[k].chars_len), dtype=np.uint8)
                    keep[k] = keep[k] + (buf,)
                    cols[k].chars, cols[k].chars_cap = buf.ctypes.data, buf.nbytes
            rc = L.lp_result_table(self._p._h, ctypes.byref(res), first, count, cols, len(columns), threads)
        if rc != LP_OK:
            raise ValueError("lp_result_table failed: %d" % rc)
        out = {}
        for k, (path, typ) in enumerate(columns):
            valid, i64, f64 = keep[k][:3]
            ok = valid[:count].astype(bool)
            if typ is str and not decode:
                out[path] = ((i64, keep[k][3] if len(keep[k]) > 3 else np.zeros(0, np.uint8)), ok)
            elif typ is str:
                chars = keep[k][3].tobytes() if len(keep[k]) > 3 else b""
                vals = [chars[i64[j]:i64[j + 1]].decode("utf-8") if ok[j] else None for j in range(count)]
                out[path] = (vals, ok)
            else:
                out[path] = ((i64[:count] if typ is int else f64[:count]).copy(), ok)
        return out

    def table_buffers(self, columns, count=None, chars_cap=None):
        """Device buffers for table_device(columns, buffers=...): per column
        [valid, i64 (STRING offsets / BIGINT values), f64 (DOUBLE), chars]
        (None where the kind has none); chars_cap: an int for every STRING
        column or {path: bytes}."""
        import torch
        count = self.n_lines if count is None else count
        dev = torch.device("cuda", self._p.device)
        keep = []
        for path, typ in columns:
            cap = chars_cap.get(path, 1) if isinstance(chars_cap, dict) else (chars_cap or 1)
            keep.append([torch.empty(max(1, count), dtype=torch.uint8, device=dev),
                         torch.empty(count + 1 if typ is str else max(1, count), dtype=torch.int64, device=dev)
                         if typ is not float else None,
                         torch.empty(max(1, count), dtype=torch.float64, device=dev) if typ is float else None,
                         torch.empty(max(1, cap), dtype=torch.uint8, device=dev) if typ is str else None])
        return keep

    def table_device(self, columns, first=0, count=None, chars_cap=None, buffers=None):
        """lp_result_table on the device view: typed columns of rows [first,
        first+count) built in HBM.  columns: [(path, str | int | float)].
        Returns {path: (values, valid)} of torch tensors on the handle's
        device: valid uint8 [count]; STRING columns the Arrow pair (offsets
        int64 [count + 1], chars uint8), BIGINT int64 / DOUBLE float64 [count].
        chars_cap: bytes allotted per STRING column (default: enough after a
        first call that reports the need); buffers: table_buffers(...) to
        fill instead of fresh ones."""
        count = self.n_lines - first if count is None else count
        kinds = {str: CAST_STRING, int: CAST_LONG, float: CAST_DOUBLE}
        res = LpResult()
        L = lib()
        rc = L.lp_result_view(self._p._h, ctypes.byref(res))
        if rc != LP_OK:
            raise EngineUnavailable("lp_result_view failed: %d" % rc)
        cols = (LpTableCol * len(columns))()
        keep = buffers if buffers is not None else self.table_buffers(columns, count, chars_cap)
        for k, (path, typ) in enumerate(columns):
            c = cols[k]
            c.path = path.encode()
            c.kind = kinds[typ]
            valid, i64, f64, chars = keep[k]
            c.valid = valid.data_ptr()
            c.i64 = i64.data_ptr() if i64 is not None else 0
            c.f64 = f64.data_ptr() if f64 is not None else 0
            if chars is not None:
                c.chars = chars.data_ptr()
                c.chars_cap = chars.numel() if (chars_cap or buffers is not None) else 0
        rc = L.lp_result_table(self._p._h, ctypes.byref(res), first, count, cols, len(columns), 0)
        if rc == LP_E_NOMEM:
            import torch
            dev = torch.device("cuda", self._p.device)
            for k, (path, typ) in enumerate(columns):
                if typ is str and cols[k].chars_len > cols[k].chars_cap:
                    keep[k][3] = torch.empty(max(1, cols[k].chars_len), dtype=torch.uint8, device=dev)
                    cols[k].chars, cols[k].chars_cap = keep[k][3].data_ptr(), keep[k][3].numel()
            rc = L.lp_result_table(self._p._h, ctypes.byref(res), first, count, cols, len(columns), 0)
        if rc == LP_E_UNSUPPORTED:
            raise FallbackRequired("a column's values are derived on the host only: use table_from")
        if rc != LP_OK:
            raise ValueError("lp_result_table (device) failed: %d" % rc)
        out = {}
        for k, (path, typ) in enumerate(columns):
            valid, i64, f64, chars = keep[k]
            if typ is str:
                out[path] = ((i64[:count + 1], chars[:cols[k].chars_len]), valid[:count])
            else:
                out[path] = ((i64 if typ is int else f64)[:count], valid[:count])
        return out

    def table_timing(self):
        """HIP-event ms of the last device lp_result_table's phases:
        {"values": k_table_values, "scans": offset scans, "chars": k_table_chars}"""
        t = (ctypes.c_float * 8)()
        lib().lp_last_timing(self._p._h, t, 8)
        return {"values": t[5], "scans": t[6], "chars": t[7]}

    def record_json_from(self, res, i):
        """lp_result_record_json: the record of line i from a host copy."""
        cap = 1 << 16
        while True:
            out = ctypes.create_string_buffer(cap)
            n = lib().lp_result_record_json(self._p._h, ctypes.byref(res), i, out, cap)
            if n >= 0:
                return out.value.decode("utf-8")
            if n <= -100:
                cap = int(-n - 100) + 16
                continue
            if n == LP_E_STATE:
                raise ValueError("line %d is not OK" % i)
            raise EngineUnavailable("lp_result_record_json failed: %d" % n)


class HttpdLoglineParser:
    """GPU-backed equivalent of new HttpdLoglineParser<>(RECORD.class, logformat)
    with addParseTarget(...) for each requested "TYPE:path"."""

    def __init__(self, logformat, fields=(), device=0, force_direct=False, reserve_lines=0, reserve_arena=0,
                 options=None):
        self.logformat = logformat
        self.fields = list(fields)
        self._targets = {}       # cleaned "TYPE:path" -> [Target] (Parser.targets)
        self._remaps = {}        # path -> {TYPE} (Parser.typeRemappings)
        self._remap_casts = {}   # "TYPE:path" -> casts of a remapped target
        self._engine_fields = None
        self.device = device
        self.force_direct = force_direct
        self.reserve = (reserve_lines, reserve_arena)
        self.options = dict(options or {})  # lp_set_option(OPT_*, value) after lp_compile
        self._h = None
        self.device_program_ok = None
        self.unsupported_reason = ""

    # Parser.addParseTarget (core/Parser.java:517-635)
    def add_parse_target(self, *fields, setter=None, setter_policy=SetterPolicy.ALWAYS, value_class=str):
        """Request fields.  With a setter (a method name of the record passed
        to parse, or a callable taking (value) or (name, value)), parse(line,
        record) delivers them through it with Parser.store's rules: value_class
        str / int / float = a String / Long / Double setter, setter_policy a
        SetterPolicy."""
        self.fields.extend(fields)
        if setter is not None:
            for f in fields:
                self._targets.setdefault(cleanup_field_value(f), []).append(Target(setter, setter_policy, value_class))
        self._close()
        return self

    # Parser.addTypeRemapping(s) / setTypeRemappings (core/Parser.java:636-677)
    def add_type_remapping(self, input_name, new_type, casts=STRING_ONLY):
        name, typ = input_name.strip().lower(), new_type.strip().upper()
        if typ not in self._remaps.setdefault(name, set()):
            self._remaps[name].add(typ)
            self._remap_casts[typ + ":" + name] = casts
        self._close()
        return self

    def add_type_remappings(self, mappings):
        for name, types in mappings.items():
            for t in types:
                self.add_type_remapping(name, t)
        return self

    def set_type_remappings(self, mappings):
        self._remaps, self._remap_casts = {}, {}
        return self.add_type_remappings(mappings or {})

    # Parser.getCasts (core/Parser.java:127-129)
    def get_casts(self, name):
        """CAST_* bits of a requested "TYPE:path" (None if unknown)"""
        name = cleanup_field_value(name)
        self._ensure()
        c = lib().lp_casts(self._h, name.encode())
        return None if c < 0 else c

    def _remap_list(self):
        """[(input, TYPE, casts)] in a stable order"""
        return [(n, t, self._remap_casts[t + ":" + n]) for n in sorted(self._remaps) for t in sorted(self._remaps[n])]

    def get_possible_paths(self, max_depth=15):
        return get_possible_paths(self.logformat, max_depth, self._remap_list())

    def _ensure(self):
        if self._h:
            return
        L = lib()
        fields = list(self.fields)
        self._engine_fields = fields
        arr = (ctypes.c_char_p * max(1, len(fields)))()
        for i, f in enumerate(fields):
            arr[i] = f.encode()
        rm, n_rm = _remap_array(self._remap_list())
        st = ctypes.c_int(0)
        err = ctypes.create_string_buffer(1024)
        h = L.lp_compile_remapped(self.logformat.encode(), arr, len(fields), rm, n_rm, self.device, ctypes.byref(st),
                                  err, 1024)
        msg = err.value.decode(errors="replace")
        if not h:
            if st.value == LP_E_MISSING:
                raise MissingDissectorsException(msg)
            if st.value == LP_E_DEVICE:
                raise EngineUnavailable(msg)
            raise InvalidDissectorException(msg)
        self._h = h
        if self.force_direct:
            L.lp_set_option(h, OPT_FORCE_DIRECT, 1)
        if self.reserve[0] or self.reserve[1]:
            L.lp_reserve(h, self.reserve[0], self.reserve[1])
        for opt, val in self.options.items():
            if L.lp_set_option(h, opt, val) != LP_OK:
                raise ValueError("lp_set_option(%r, %r) rejected" % (opt, val))
        self.device_program_ok = st.value == LP_OK
        self.unsupported_reason = msg if st.value == LP_E_UNSUPPORTED else ""

    def parse_batch(self, data, stream=None):
        """Parse every '\\n'-separated line.  data: bytes / bytearray / numpy
        uint8 (host, copied to HBM) or a torch.uint8 CUDA tensor (in HBM)."""
        self._ensure()
        L = lib()
        s = ctypes.c_void_p(stream) if stream is not None else None
        if hasattr(data, "data_ptr") and getattr(data, "is_cuda", False):
            rc = L.lp_parse_batch(self._h, ctypes.c_void_p(data.data_ptr()), data.numel() * data.element_size(),
                                  BUF_DEVICE, s)
        else:
            if isinstance(data, np.ndarray):
                buf = np.ascontiguousarray(data, dtype=np.uint8)
                ptr, n = buf.ctypes.data, buf.nbytes
            else:
                buf = bytes(data)
                ptr, n = ctypes.cast(ctypes.c_char_p(buf), ctypes.c_void_p).value, len(buf)
            rc = L.lp_parse_batch(self._h, ctypes.c_void_p(ptr), n, BUF_HOST, s)
            L.lp_sync(self._h)  # the host buffer must outlive the copy
        if rc != LP_OK:
            raise EngineUnavailable("lp_parse_batch failed: %d" % rc)
        return BatchResult(self)

    def histograms(self, device_ptr=None):
        """lp_histograms of the last batch: the 1024 u64 words (numpy) in host
        memory, or written to device_ptr (a device buffer of 8 KiB on the
        handle's device, e.g. a torch tensor to all-reduce) when given"""
        self._ensure()
        if device_ptr is not None:
            rc = lib().lp_histograms(self._h, ctypes.c_void_p(device_ptr), 1)
            if rc != LP_OK:
                raise EngineUnavailable("lp_histograms failed: %d" % rc)
            return None
        out = np.zeros(HIST_WORDS, dtype=np.uint64)
        rc = lib().lp_histograms(self._h, out.ctypes.data, 0)
        if rc != LP_OK:
            raise EngineUnavailable("lp_histograms failed: %d" % rc)
        return out

    def run(self, data_ptr, nbytes, on_device=True, stream=None):
        """Lean batch call for benchmarks/pipelines: parse nbytes at data_ptr
        (a device pointer when on_device), wait, and return the device
        counters, HIP-event timings and algorithmic byte counts (no per-line
        copies to the host)."""
        self._ensure()
        L = lib()
        rc = L.lp_parse_batch(self._h, ctypes.c_void_p(data_ptr), nbytes, BUF_DEVICE if on_device else BUF_HOST,
                              ctypes.c_void_p(stream) if stream is not None else None)
        if rc != LP_OK:
            raise EngineUnavailable("lp_parse_batch failed: %d" % rc)
        rc = L.lp_sync(self._h)
        if rc != LP_OK:
            raise EngineUnavailable("lp_sync failed: %d" % rc)
        c = (ctypes.c_uint64 * 9)()
        L.lp_counters(self._h, c, 9)
        t = (ctypes.c_float * 5)()
        L.lp_last_timing(self._h, t, 5)
        b = (ctypes.c_uint64 * 4)()
        L.lp_last_bytes(self._h, b, 4)
        return {"lines": c[0], "ok": c[1], "bad": c[2], "fallback": c[3], "overflow_waves": c[4], "retries": c[5],
                "arena_ovf": c[6], "uri_overflow_waves": c[7], "deferred_chunks": c[8],
                "ms_total": t[0], "ms_index": t[1], "ms_parse": t[2], "ms_parse_kernels": t[3], "ms_uri_kernels": t[4],
                "bytes_in": b[0], "bytes_out": b[1], "bytes_parse_kernels": b[2], "bytes_uri_kernels": b[3]}

    def parse(self, line, record=None):
        """Parser.parse(line) / parse(record, line) (core/Parser.java:700-756):
        without setters the record's values as {"TYPE:path": [values]}; with
        setters (add_parse_target(..., setter=...)) the values are delivered
        into `record` through them and `record` is returned.
        DissectionFailure for a bad line, FallbackRequired when the device
        cannot prove the line."""
        if isinstance(line, str):
            line = line.encode("utf-8")
        if b"\n" in line:
            raise ValueError("one line without terminator expected")
        r = self.parse_batch(line)
        if r.n_lines != 1:
            raise DissectionFailure("empty input")
        if r.status[0] == LINE_BAD:
            raise DissectionFailure("The input line does not match the specified log format.")
        if r.status[0] == LINE_FALLBACK:
            raise FallbackRequired(self.unsupported_reason or "line outside the device's proven subset")
        if not self._targets:
            return r.record(0)
        _, res = r.copy_to_host()
        return self.deliver(r.emissions_from(res, 0), record)

    def deliver(self, emissions, record):
        """Parser.store of one line's emissions (BatchResult.emissions_from)
        into `record` through the registered setters"""
        casts = {}

        def cast_of(name):
            if name not in casts:
                casts[name] = self.get_casts(name)
            return casts[name]
        return deliver(emissions, record, self._targets, cast_of, self._remaps)

    def describe(self):
        self._ensure()
        out = ctypes.create_string_buffer(1 << 16)
        lib().lp_describe(self._h, out, 1 << 16)
        return out.value.decode()

    def _close(self):
        if self._h:
            lib().lp_free(self._h)
            self._h = None

    def __del__(self):
        try:
            self._close()
        except Exception:
            pass


# lp_histograms layout (include/logparser_amd.h)
HIST_WORDS = 1024
HIST_METHODS = ["GET", "POST", "HEAD", "PUT", "DELETE", "OPTIONS", "PATCH", "CONNECT", "TRACE", "PROPFIND", "MKCOL",
                "COPY", "MOVE", "LOCK", "UNLOCK", "(other)", "(none)"]


def decode_histograms(h):
    """the words of lp_histograms (or their all-reduced sum) as a dict"""
    h = [int(x) for x in h]
    return {
        "lines": h[0], "ok": h[1], "bad": h[2], "fallback": h[3],
        "token_null": h[16:32], "token_present": h[32:48],
        "status_other": h[48],
        "methods": {m: h[64 + i] for i, m in enumerate(HIST_METHODS) if h[64 + i]},
        "status": {c: h[100 + c] for c in range(100, 600) if h[100 + c]},
    }
