"""GPU parity: the HIP path (through the C ABI) against the oracle on the same
inputs -- reference golden vectors, the reference demo log, synthetic
config-2 lines, mutated/malformed lines, edge cases -- plus size-independent
properties at a large batch size."""
import json
import random

import numpy as np
import pytest

import golden_check
import logparser_amd as lpa

pytestmark = pytest.mark.gpu

_PATHS = {}


def paths(oracle, fmt="combined"):
    if fmt not in _PATHS:
        _PATHS[fmt] = oracle.possible_paths(fmt)
    return _PATHS[fmt]


def gpu_vs_oracle(oracle, fmt, fields, lines, allow_fallback=True, data=None, remaps=()):
    """lines: the expected lines; data: the batch buffer (default: the lines + '\n');
    remaps: [(input, TYPE)] type remappings of both parsers"""
    p = lpa.HttpdLoglineParser(fmt, fields)
    for name, typ in remaps:
        p.add_type_remapping(name, typ)
    if data is None:
        data = b"".join(l + b"\n" for l in lines)
    r = p.parse_batch(data)
    assert r.n_lines == len(lines)
    o = oracle.Oracle(fmt, fields, remaps)
    stats = {"ok": 0, "bad": 0, "fallback": 0}
    for i, l in enumerate(lines):
        s2 = int(r.status[i])
        s1, r1 = o.parse_raw(l)
        if s2 == lpa.LINE_FALLBACK:
            stats["fallback"] += 1
            assert allow_fallback, l
            continue
        assert s1 != oracle.UNSUPPORTED, l
        assert s1 == s2, (i, l, s1, s2)
        if s1 == oracle.OK:
            r2 = r.record_json(i)
            assert r1 == r2, (l, r1[:1500], r2[:1500])
            stats["ok"] += 1
        else:
            stats["bad"] += 1
    c = r.counters
    assert c["lines"] == len(lines)
    assert c["ok"] == stats["ok"] and c["bad"] == stats["bad"] and c["fallback"] == stats["fallback"]
    return stats, r


def test_golden_vectors_gpu(oracle, vectors):
    groups = {}
    for c in vectors["cases"]:
        groups.setdefault((c["logformat"], tuple(c["fields"]), tuple(map(tuple, c["remaps"]))), []).append(c)
    checked, fallback, unsupported = 0, [], 0
    for (fmt, fields, remaps), cases in groups.items():
        p = lpa.HttpdLoglineParser(fmt, list(fields))
        for name, typ in remaps:
            p.add_type_remapping(name, typ)
        data = b"".join(c["line"].encode() + b"\n" for c in cases)
        r = p.parse_batch(data)
        assert r.n_lines == len(cases)
        if not p.device_program_ok:
            unsupported += len(cases)
        for i, c in enumerate(cases):
            st = int(r.status[i])
            if st == lpa.LINE_FALLBACK:
                fallback.append(c["source"])
                continue
            rec = r.record(i) if st == lpa.LINE_OK else {}
            assert golden_check.check_case(c, st, rec) == [], c["source"]
            checked += 1
    n = len(vectors["cases"])
    print("golden vectors on the device: %d of %d (FALLBACK %d, of which %d from handles needing a "
          "dissector not on the device)" % (checked, n, len(fallback), unsupported))
    for src in sorted(set(fallback)):
        print("  FALLBACK:", src)
    assert checked >= 156, (checked, n)  # 158 of 165 in the CPU emulation of the same device code


def test_setup_vectors_gpu(vectors):
    """lp_compile refuses the requests the reference refuses (MissingDissectorsException)."""
    for c in vectors["setup_cases"]:
        with pytest.raises(lpa.MissingDissectorsException) as ei:
            lpa.HttpdLoglineParser(c["logformat"], c["fields"]).parse_batch(b"x\n")
        assert c["message_contains"] in str(ei.value), c["source"]


def test_demolog_gpu(oracle, demolog_lines):
    s, _ = gpu_vs_oracle(oracle, "combined", paths(oracle), demolog_lines)
    assert s["ok"] + s["fallback"] == 3456 and s["fallback"] < 30, s


def test_synthetic_gpu(oracle):
    lines = lpa.synth_combined(20261015, 0, 20000).split(b"\n")[:-1]
    s, _ = gpu_vs_oracle(oracle, "combined", paths(oracle), lines, allow_fallback=False)
    assert s["ok"] == 20000


def test_mutated_gpu(oracle):
    from test_emu_parity import mutate
    rng = random.Random(77)
    lines = [mutate(rng, l) for l in lpa.synth_combined(5, 0, 3000).split(b"\n")[:-1]]
    s, _ = gpu_vs_oracle(oracle, "combined", paths(oracle), lines)
    assert s["bad"] > 200 and s["ok"] > 200, s


def test_edge_cases_gpu(oracle):
    lines = [
        b"",                                       # empty line
        b"-",
        b'1.2.3.4 - - [29/Feb/2016:23:59:59 +1800] "GET / HTTP/1.1" 200 - "-" "-"',
        b'1.2.3.4 - - [29/Feb/2015:23:59:59 -1800] "GET / HTTP/1.1" 200 0 "-" "-"',   # clamp to 28 Feb
        b'1.2.3.4 - - [31/Dec/2012:24:00:00 +0000] "GET / HTTP/1.1" 200 0 "-" "-"',   # end of day
        b'1.2.3.4 - - [31/Dec/2012:24:00:01 +0000] "GET / HTTP/1.1" 200 0 "-" "-"',
        b'1.2.3.4 - - [31/Dec/2012:23:00:00 +1801] "GET / HTTP/1.1" 200 0 "-" "-"',
        b'1.2.3.4 - - [31/Dec/2012:23:00:00 |0100] "GET / HTTP/1.1" 200 0 "-" "-"',
        b'1.2.3.4 - - [01/Jan/2021:00:00:00 +0000] "GET  HTTP/1.1" 200 0 "-" "-"',
        b'1.2.3.4 - - [01/Jan/2021:00:00:00 +0000] "GET HTTP/1.1" 200 0 "-" "-"',
        b'1.2.3.4 - - [01/Jan/2021:00:00:00 +0000] "" 200 0 "" ""',
        b'1.2.3.4 - - [01/Jan/2021:00:00:00 +0000] "GET /x" y" 200 0 "a" "b" "c"',
        b'1.2.3.4 - - [01/Jan/2021:00:00:00 +0000] "GET /?a=1&B=%41%C3%A9+x&=v&c HTTP/1.1" 200 0 "http://h:99/p?q=1#f" "u"',
        b'1.2.3.4 - - [01/Jan/2021:00:00:00 +0000] "GET /%C3%A9 HTTP/1.1" 200 0 "http://under_score.example.com/" "u"',
        b'1.2.3.4 - - [01/Jan/2021:00:00:00 +0000] "GET / HTTP/1.1" 200 0 "http://1.2.3.4.5/" "u"',
        b'1.2.3.4 - - [01/Jan/2021:00:00:00 +0000] "GET / HTTP/1.1" 200 0 "http://h:99999999999/" "u"',
        b'1.2.3.4 - - [01/Jan/2021:00:00:00 +0000] "GET / HTTP/1.1" 200 0 "foo bar:baz" "u"',
        b'1.2.3.4 - - [01/Jan/2021:00:00:00 +0000] "GET / HTTP/1.1" 200 0 "relative/path?x" "u"',
        b'1.2.3.4 - - [01/Jan/2021:00:00:00 +0000] "GET / HTTP/1.1" 200 0 "http:/abs?x" "u"',
        b'1.2.3.4 - - [01/Jan/2021:00:00:00 +0000] "GET / HTTP/1.1" 200 0 "-" "u" trailing',
        b"x" * 9000,                               # longer than the device window
    ]
    gpu_vs_oracle(oracle, "combined", paths(oracle), lines)


def test_no_trailing_newline_and_batches(oracle):
    p = lpa.HttpdLoglineParser("combined", ["IP:connection.client.host", "TIME.EPOCH:request.receive.time.epoch"])
    lines = lpa.synth_combined(11, 0, 1000).split(b"\n")[:-1]
    r1 = p.parse_batch(b"\n".join(lines))          # last line unterminated
    assert r1.n_lines == 1000 and r1.counters["ok"] == 1000
    last = r1.record(999)
    r2 = p.parse_batch(lines[-1] + b"\n")
    assert r2.n_lines == 1 and r2.record(0) == last
    r3 = p.parse_batch(b"")
    assert r3.n_lines == 0


def test_device_tensor_input(oracle):
    import torch
    lines = lpa.synth_combined(12, 0, 2000)
    t = torch.from_numpy(np.frombuffer(lines, dtype=np.uint8).copy()).cuda()
    p = lpa.HttpdLoglineParser("combined", paths(oracle))
    a = p.parse_batch(t)
    recs = [a.record_json(i) for i in range(0, 2000, 97)]
    b = p.parse_batch(lines)
    assert [b.record_json(i) for i in range(0, 2000, 97)] == recs
    # a line-aligned slice that starts mid-word (a batch of a larger buffer)
    for skew in (1, 3, 7, 13):
        u = torch.zeros(len(lines) + 16, dtype=torch.uint8, device="cuda")
        u[skew:skew + len(lines)].copy_(t)
        c = p.parse_batch(u[skew:skew + len(lines)])
        assert c.n_lines == 2000 and c.counters["ok"] == 2000
        assert [c.record_json(i) for i in range(0, 2000, 97)] == recs


def test_large_batch_properties(oracle):
    """2M synthetic lines: every line OK (no FALLBACK on config-2 data), the
    line index matches the newline count, and a deterministic sample of
    lines matches the oracle exactly."""
    n = 2_000_000
    data = lpa.synth_combined(20261015, 0, n)
    p = lpa.HttpdLoglineParser("combined", paths(oracle))
    r = p.parse_batch(data)
    assert r.n_lines == n == data.count(b"\n")
    assert r.counters == {"lines": n, "ok": n, "bad": 0, "fallback": 0}
    o = oracle.Oracle("combined", paths(oracle))
    rng = random.Random(3)
    for i in sorted(rng.sample(range(n), 300)):
        a = r.line_offset(i)
        b = r.line_offset(i + 1) - 1
        line = data[a:b]
        s1, js = o.parse_raw(line)
        assert s1 == 0 and js == r.record_json(i), i


def test_headline_parity_every_line(oracle):
    """Whole-batch parity at headline scale: EVERY line of a 10 M-line
    config-2 batch (2.5 GB, all 123 paths) against the oracle.  Both sides
    reduce a line to (status, FNV-1a of its canonical JSON record) on 16
    host threads (oracle/digest.c); the engine side replays its records from
    one lp_result_copy of the batch, through lp_result_record_json."""
    import ctypes
    import os
    n = int(os.environ.get("LP_HEADLINE_LINES", "10000000"))
    threads = 16
    fields = paths(oracle)
    data = lpa.synth_combined(20261015, 0, n)
    p = lpa.HttpdLoglineParser("combined", fields)
    r = p.parse_batch(data)
    assert r.n_lines == n
    assert r.counters == {"lines": n, "ok": n, "bad": 0, "fallback": 0}
    buf, res = r.copy_to_host(with_input=True)
    fn = ctypes.cast(lpa.lib().lp_result_record_json, ctypes.c_void_p).value
    h_eng = oracle.digest_engine(fn, p._h, ctypes.addressof(res), r.status, threads)
    st_orc, h_orc = oracle.digest_lines("combined", fields, data, threads, n + 1)
    assert len(st_orc) == n
    assert np.array_equal(st_orc, r.status.astype(np.uint8))
    diff = np.nonzero(h_eng != h_orc)[0]
    assert len(diff) == 0, (len(diff), diff[:10].tolist())
    assert np.count_nonzero(h_eng) == n  # every line produced a record


def _newline_batches(data, batch_bytes):
    """[(start, end)) pieces of about batch_bytes, each cut just after a '\\n'
    (bench.newline_batches on a host buffer)"""
    out, a = [], 0
    while len(data) - a > batch_bytes:
        c = data.index(b"\n", a + batch_bytes) + 1
        out.append((a, c))
        a = c
    if a < len(data):
        out.append((a, len(data)))
    return out


@pytest.mark.parametrize("workload", [3, 4, 5])
def test_every_line_parity_other_configs(oracle, workload):
    """Every line of a 2 M-line batch of BASELINE configs 3, 4 and 5 against
    the oracle, by (status, FNV-1a of the record) digests on 16 host threads
    (oracle/digest.c): config 3 with its 5 % malformed lines (status BAD must
    agree line by line), config 4's NGINX upstream format, and config 5's
    three-format corpus streamed through ONE handle in newline-aligned 48 MiB
    batches (about 10), so the sticky routing state crosses batches as in the
    timed bench run (the oracle side: one parser per thread, each warmed up
    on the 2000 lines before its range, digest.c).  No FALLBACK is allowed
    on these workloads (configs 3-5 are inside the device subset)."""
    import ctypes
    import os
    seeds = {3: 20261016, 4: 20261017, 5: 20261018}
    n = int(os.environ.get("LP_OTHER_CONFIG_LINES", "2000000"))
    threads = 16
    fmt = lpa.SYNTH_FORMATS[workload]
    fields = paths(oracle, fmt)
    data = lpa.synth(workload, seeds[workload], 0, n)
    assert data.count(b"\n") == n
    p = lpa.HttpdLoglineParser(fmt, fields)
    fn = ctypes.cast(lpa.lib().lp_result_record_json, ctypes.c_void_p).value
    pieces = _newline_batches(data, 48 << 20) if workload == 5 else [(0, len(data))]
    if workload == 5:
        assert len(pieces) >= 8
    st_eng, h_eng = [], []
    for a, b in pieces:
        r = p.parse_batch(data[a:b])
        assert r.n_lines == data.count(b"\n", a, b)
        assert r.counters["fallback"] == 0, r.counters
        buf, res = r.copy_to_host(with_input=True)
        st_eng.append(r.status.astype(np.uint8).copy())
        h_eng.append(oracle.digest_engine(fn, p._h, ctypes.addressof(res), r.status, threads))
        del buf, res
    st_eng, h_eng = np.concatenate(st_eng), np.concatenate(h_eng)
    st_orc, h_orc = oracle.digest_lines(fmt, fields, data, threads, n + 1, warmup=2000 if workload == 5 else 0)
    assert len(st_orc) == n == len(st_eng)
    bad = np.nonzero(st_orc != st_eng)[0]
    assert len(bad) == 0, (len(bad), bad[:10].tolist(), st_orc[bad[:10]].tolist(), st_eng[bad[:10]].tolist())
    diff = np.nonzero(h_eng != h_orc)[0]
    assert len(diff) == 0, (len(diff), diff[:10].tolist())
    n_ok = int(np.count_nonzero(st_eng == oracle.OK))
    assert np.count_nonzero(h_eng) == n_ok
    if workload == 3:  # the malformed 5 % are BAD on both sides
        assert 0.03 * n < n - n_ok < 0.07 * n, n - n_ok
    else:
        assert n_ok == n


@pytest.mark.parametrize("staged", [True, False])
def test_offsets_beyond_4gb(oracle, staged):
    """A 4.4 GB batch (a 1 MB block of synthetic lines repeated on the device):
    every line OK, and lines stored past the 4 GiB mark match the oracle --
    with the LDS-window path and with the direct-HBM path (LP_OPT_FORCE_DIRECT)."""
    import torch
    block = lpa.synth_combined(31, 0, 4096)
    reps = 4_400_000_000 // len(block) + 1
    dev = torch.frombuffer(bytearray(block), dtype=torch.uint8).cuda().repeat(reps)
    p = lpa.HttpdLoglineParser("combined", paths(oracle), force_direct=not staged)
    r = p.parse_batch(dev)
    n = 4096 * reps
    assert r.n_lines == n
    assert r.counters == {"lines": n, "ok": n, "bad": 0, "fallback": 0}
    lines = block.split(b"\n")[:-1]
    o = oracle.Oracle("combined", paths(oracle))
    rng = random.Random(9)
    first_past = (2 ** 32 // len(block) + 1) * 4096
    for i in sorted(rng.sample(range(first_past, n), 40)):
        assert r.line_offset(i) >= 2 ** 32
        s1, js = o.parse_raw(lines[i % 4096])
        assert s1 == 0 and js == r.record_json(i), i
    del dev
    torch.cuda.empty_cache()


def test_nginx_config4_gpu(oracle):
    """BASELINE config 4: the NGINX log_format of NginxUpstreamTest.java:94,
    all possible paths (upstream lists, SECOND_MILLIS -> ms / us, query)."""
    from test_emu_parity import NGINX, mutate, mutate_nginx
    fields = paths(oracle, NGINX)
    lines = lpa.synth(lpa.SYNTH_NGINX, 20261017, 0, 20000).split(b"\n")[:-1]
    s, _ = gpu_vs_oracle(oracle, NGINX, fields, lines, allow_fallback=False)
    assert s["ok"] == 20000
    rng = random.Random(78)
    mut = [mutate_nginx(rng, l) for l in lines[:3000]] + [mutate(rng, l) for l in lines[3000:6000]]
    s, _ = gpu_vs_oracle(oracle, NGINX, fields, mut)
    assert s["bad"] > 100 and s["ok"] > 1000, s


def test_strftime_config3_gpu(oracle):
    """BASELINE config 3: 'combinedio' with %{%d/%b/%Y %T}t.%{msec_frac}t and
    5 % malformed lines, all possible paths (StrfTimeStampDissector on the device)."""
    from test_emu_parity import STRF, mutate, mutate_strf
    fields = paths(oracle, STRF)
    lines = lpa.synth(lpa.SYNTH_STRFTIME, 20261016, 0, 20000).split(b"\n")[:-1]
    s, _ = gpu_vs_oracle(oracle, STRF, fields, lines, allow_fallback=False)
    assert s["ok"] > 18500 and s["bad"] > 500, s
    rng = random.Random(34)
    mut = [mutate_strf(rng, l) for l in lines[:3000] if b"[" in l and len(l) > 60] + [mutate(rng, l) for l in lines[3000:6000]]
    s, _ = gpu_vs_oracle(oracle, STRF, fields, mut)
    assert s["bad"] > 300 and s["ok"] > 1000, s


@pytest.mark.parametrize("one_pass", [1, 0])
def test_mixed_formats_gpu(oracle, one_pass):
    """Sticky multi-format routing on the device against the stateful oracle
    on a mixed corpus (formats that are not mutually exclusive, mutated lines),
    across routing chunks and across two batches of one handle: one pass
    (routing inside the chunk kernel, the lines several formats match after
    the scan) and the index / routing / parse passes (LP_OPT_ONE_PASS 0)."""
    from test_emu_parity import MIXED, mixed_lines, mutate
    fields = paths(oracle, MIXED)
    rng = random.Random(57)
    lines = [mutate(rng, l) if rng.random() < 0.05 else l for l in mixed_lines(30000, 58)]
    p = lpa.HttpdLoglineParser(MIXED, fields, options={lpa.OPT_ONE_PASS: one_pass})
    o = oracle.Oracle(MIXED, fields)
    for part in (lines[:17000], lines[17000:]):
        r = p.parse_batch(b"".join(l + b"\n" for l in part))
        assert r.n_lines == len(part)
        ok = 0
        for i, l in enumerate(part):
            s1, r1 = o.parse_raw(l)
            s2 = int(r.status[i])
            if s2 == lpa.LINE_FALLBACK:
                continue
            assert s1 == s2, (i, l, s1, s2)
            if s1 == oracle.OK:
                assert r1 == r.record_json(i), (i, l)
                ok += 1
        assert ok > 0.8 * len(part)


def test_authority_variants_gpu(oracle):
    from test_emu_parity import HOSTS
    base = b'1.2.3.4 - - [01/Jan/2021:00:00:00 +0000] "GET / HTTP/1.1" 200 0 "http://%s/p?q=1" "u"'
    lines = [base.replace(b"%s/p?q=1", (h + t + "/p?q=1").encode()) for h in HOSTS for t in ("", "/x", "#f", "?a")]
    s, _ = gpu_vs_oracle(oracle, "combined", paths(oracle), lines)
    assert s["ok"] > 100, s


def test_mixed_config5_gpu(oracle):
    """BASELINE config 5: the mixed-format corpus (lp_synth workload 5) through
    one three-format handle, bit-exact against the stateful oracle with no
    FALLBACK; then the same lines streamed as three batches of one handle
    (routing state carried across batches, as bench.py --workload 5 does)
    give the same statuses and records."""
    fmt = lpa.SYNTH_FORMATS[lpa.SYNTH_MIXED]
    fields = paths(oracle, fmt)
    lines = lpa.synth(lpa.SYNTH_MIXED, 20261018, 0, 20000).split(b"\n")[:-1]
    s, r = gpu_vs_oracle(oracle, fmt, fields, lines, allow_fallback=False)
    assert s["ok"] == 20000, s
    whole = [r.record_json(i) for i in range(0, 20000, 97)]
    p = lpa.HttpdLoglineParser(fmt, fields)
    got = {}
    base = 0
    for part in (lines[:6001], lines[6001:13333], lines[13333:]):
        rb = p.parse_batch(b"".join(l + b"\n" for l in part))
        assert rb.n_lines == len(part) and rb.counters["ok"] == len(part)
        for i in range(len(part)):
            if (base + i) % 97 == 0:
                got[base + i] = rb.record_json(i)
        base += len(part)
    assert [got[i] for i in range(0, 20000, 97)] == whole


@pytest.mark.parametrize("which", ["nginx", "mixed"])
def test_ip_token_variants_gpu(oracle, which):
    """Non-IPv4 hosts in FORMAT_IP / FORMAT_CLF_IP tokens: the DFS's exact
    resolution of the IPv6 branch's other ends (nested DFS) on the device."""
    from test_emu_parity import IP_TOKENS, MIXED, NGINX
    fmt = {"nginx": NGINX, "mixed": MIXED}[which]
    base = lpa.synth(lpa.SYNTH_MIXED, 20261018, 0, 60).split(b"\n")[:-1]
    lines = [t.encode() + b" " + l.split(b" ", 1)[1] for l in base for t in IP_TOKENS[:: 1 + len(l) % 3]]
    if which == "nginx":
        s, _ = gpu_vs_oracle(oracle, fmt, paths(oracle, fmt), lines)
        assert s["fallback"] < len(lines) // 4 and s["bad"] > len(lines) // 2, s
    else:  # stateful routing: compare line by line against the sticky oracle
        fields = paths(oracle, fmt)
        r = lpa.HttpdLoglineParser(fmt, fields).parse_batch(b"".join(l + b"\n" for l in lines))
        o = oracle.Oracle(fmt, fields)
        fb = 0
        for i, l in enumerate(lines):
            s1, r1 = o.parse_raw(l)
            s2 = int(r.status[i])
            if s2 == lpa.LINE_FALLBACK:
                fb += 1
                continue
            assert s1 == s2, (i, l, s1, s2)
            if s1 == oracle.OK:
                assert r1 == r.record_json(i), (i, l)
        assert fb < len(lines) // 4, fb


def test_bulk_results_rebuild_records(oracle):
    """lp_result_copy hands the whole batch's SoA to the host in one call;
    records rebuilt from that copy alone (lp_result_record_json) are byte-
    identical to lp_line_record_json for every line of a 100 k-line batch, and
    a 1 M-line batch's copy is consistent (line index, statuses, spans) with
    the input, with a sample of its records equal to the oracle's."""
    fields = paths(oracle)
    p = lpa.HttpdLoglineParser("combined", fields)
    data = lpa.synth_combined(20261015, 0, 100_000)
    r = p.parse_batch(data)
    buf, res = r.copy_to_host()
    assert res.n_lines == 100_000 and res.on_host == 1
    for i in range(res.n_lines):
        assert r.record_json_from(res, i) == r.record_json(i), i
    # 1 M lines: the bulk copy alone
    n = 1_000_000
    data = lpa.synth_combined(77, 0, n)
    r = p.parse_batch(data)
    buf, res = r.copy_to_host()
    cols = r.columns(res)
    assert res.n_lines == n
    off = np.ctypeslib.as_array((ctypes_u64 * (n + 1)).from_address(res.line_off))
    nl = np.flatnonzero(np.frombuffer(data, dtype=np.uint8) == 10)
    assert np.array_equal(off[1:], nl + 1) and off[0] == 0
    assert (cols[("status", 0)] == 0).all()
    lens = (off[1:] - off[:-1] - 1).astype(np.int64)
    for k in range(9):
        sp = cols[("tok_span", k)].astype(np.int64)
        assert ((sp >> 16) <= lens).all() and ((sp & 0xFFFF) <= (sp >> 16)).all()
    o = oracle.Oracle("combined", fields)
    lines = data.split(b"\n")
    rng = random.Random(5)
    for i in sorted(rng.sample(range(n), 2000)):
        s1, js = o.parse_raw(lines[i])
        assert s1 == 0 and js == r.record_json_from(res, i), i


ctypes_u64 = __import__("ctypes").c_uint64


def test_arena_overflow_retry(oracle):
    """Query-dense (beacon-style) lines need far more arena than the first
    batch's estimate: the shards overflow, lp_sync re-runs the batch with an
    exact arena, and every line matches the oracle."""
    fields = paths(oracle)
    q = "&".join("k%d=v%%41%d+x" % (j, j) for j in range(40))
    lines = [('10.0.0.%d - - [01/Jan/2021:00:00:%02d +0000] "GET /b?%s HTTP/1.1" 200 1 "http://h.nl/r?%s" "u"'
              % (i % 250, i % 60, q, q)).encode() for i in range(20000)]
    s, r = gpu_vs_oracle(oracle, "combined", fields, lines, allow_fallback=False)
    assert s["ok"] == 20000


def _query_lines(n):
    q = "&".join("k%d=v%%41%d+x" % (j, j) for j in range(12))
    return [('10.0.0.%d - - [01/Jan/2021:00:00:%02d +0000] "GET /b?%s HTTP/1.1" 200 1 "http://h.nl/r?%s" "u"'
             % (i % 250, i % 60, q, q)).encode() for i in range(n)]


def test_tiny_arena_reruns(oracle):
    """A first run with a far too small arena (LP_OPT_ARENA_BYTES) is re-run
    inside lp_sync with the exact size: LP_OK, retries > 0, every line equals
    the oracle (re-runs must not keep the short reservation)."""
    fields = paths(oracle)
    lines = _query_lines(20000)
    p = lpa.HttpdLoglineParser("combined", fields, reserve_arena=4096, options={lpa.OPT_ARENA_BYTES: 64 * 1024})
    r = p.parse_batch(b"".join(l + b"\n" for l in lines))
    assert r.diag["retries"] > 0 and r.diag["arena_ovf"] == 0, r.diag
    assert r.counters["ok"] == len(lines)
    o = oracle.Oracle("combined", fields)
    for i in range(0, len(lines), 97):
        s1, js = o.parse_raw(lines[i])
        assert s1 == oracle.OK and js == r.record_json(i), i


def test_arena_overflow_degrades_to_fallback(oracle):
    """No re-runs allowed and a tiny arena: the batch is still delivered
    (LP_OK); the lines whose arena region or query pieces did not fit are
    FALLBACK, every other line equals the oracle."""
    fields = paths(oracle)
    heavy = _query_lines(20000)
    # a quarter query-heavy lines (they need the arena), the rest plain (no arena)
    lines = [heavy[i] if i % 4 == 0 else
             b'10.1.2.3 - - [01/Jan/2021:00:00:00 +0000] "GET /plain/%d.html HTTP/1.1" 200 1 "-" "u"' % i
             for i in range(20000)]
    p = lpa.HttpdLoglineParser("combined", fields, options={lpa.OPT_MAX_RETRIES: 0, lpa.OPT_ARENA_BYTES: 1 << 20})
    r = p.parse_batch(b"".join(l + b"\n" for l in lines))
    c = r.counters
    assert r.diag["retries"] == 0 and r.diag["arena_ovf"] > 0, r.diag
    assert c["fallback"] > 0 and c["ok"] > 0 and c["ok"] + c["fallback"] == len(lines), c
    assert int((r.status == lpa.LINE_FALLBACK).sum()) == c["fallback"]
    o = oracle.Oracle("combined", fields)
    for i in range(len(lines)):
        if r.status[i] == lpa.LINE_OK and (i % 7 == 0 or r.status[max(0, i - 1)] != lpa.LINE_OK):
            s1, js = o.parse_raw(lines[i])
            assert s1 == oracle.OK and js == r.record_json(i), i
    print("arena degrade: %d of %d lines FALLBACK, %d overflow events" % (c["fallback"], len(lines), r.diag["arena_ovf"]))


def test_first_line_numbers(oracle):
    """lp_parse_batch_at numbers a batch's lines from first_line_no (a split
    reader's position); lp_parse_batch continues the handle's numbering; the
    number comes back in lp_result.first_line."""
    import ctypes
    L = lpa.lib()
    data = lpa.synth_combined(5, 0, 1000)
    t = __import__("torch").frombuffer(bytearray(data), dtype=__import__("torch").uint8).cuda()
    p = lpa.HttpdLoglineParser("combined", ["IP:connection.client.host"])
    p._ensure()
    res = lpa.LpResult()
    assert L.lp_parse_batch_at(p._h, ctypes.c_void_p(t.data_ptr()), len(data), 123456789, lpa.BUF_DEVICE, None) == 0
    assert L.lp_sync(p._h) == 0 and L.lp_result_view(p._h, ctypes.byref(res)) == 0
    assert res.first_line == 123456789 and res.n_lines == 1000
    assert L.lp_parse_batch(p._h, ctypes.c_void_p(t.data_ptr()), len(data), lpa.BUF_DEVICE, None) == 0
    assert L.lp_sync(p._h) == 0 and L.lp_result_view(p._h, ctypes.byref(res)) == 0
    assert res.first_line == 123456789 + 1000
    buf = bytearray(-L.lp_result_copy(p._h, None, 0, 0, None))
    host = (ctypes.c_uint8 * len(buf)).from_buffer(buf)
    assert L.lp_result_copy(p._h, host, len(buf), 0, ctypes.byref(res)) > 0 and res.first_line == 123456789 + 1000
    assert L.lp_parse_batch_at(p._h, None, 0, -1, lpa.BUF_DEVICE, None) == lpa.LP_E_INVALID


def test_async_batches_and_capacity_retry(oracle):
    """Later batches of a handle are enqueued without a line count (capacity
    from the previous batch); a batch of much shorter lines outgrows the
    columns and is re-run inside lp_sync; a reservation makes even the first
    batch asynchronous.  Results equal the oracle throughout."""
    fields = ["IP:connection.client.host", "TIME.EPOCH:request.receive.time.epoch", "HTTP.PATH:request.firstline.uri.path"]
    o = oracle.Oracle("combined", fields)
    long_lines = [l + b" " * 0 for l in lpa.synth_combined(3, 0, 5000).split(b"\n")[:-1]]
    short = [b'1.2.3.4 - - [01/Jan/2021:00:00:00 +0000] "GET /%d HTTP/1.1" 200 1 "-" "u"' % i for i in range(60000)]
    for reserve in (0, 100000):
        p = lpa.HttpdLoglineParser("combined", fields, reserve_lines=reserve)
        for batch in (long_lines, short, long_lines[:10], short):
            r = p.parse_batch(b"".join(l + b"\n" for l in batch))
            assert r.n_lines == len(batch) and r.counters["ok"] == len(batch)
            for i in range(0, len(batch), 997):
                s1, js = o.parse_raw(batch[i])
                assert s1 == 0 and js == r.record_json(i)


def test_result_emit_replays_setter_calls(oracle):
    """lp_result_emit gives, per line, the (base, type, name, value)
    addDissection calls a Java GpuHttpdLogFormatDissector replays
    (core/Parsable.java:142-193): rebuilding the record from them with the
    reference's exact / wildcard rule gives the record of lp_line_record_json."""
    import json
    for fmt in ("combined", lpa.SYNTH_FORMATS[lpa.SYNTH_NGINX]):
        fields = paths(oracle, fmt)
        wl = lpa.SYNTH_COMBINED if fmt == "combined" else lpa.SYNTH_NGINX
        p = lpa.HttpdLoglineParser(fmt, fields)
        r = p.parse_batch(lpa.synth(wl, 9, 0, 3000))
        _, res = r.copy_to_host()
        need = set(fields)
        for i in range(0, 3000, 7):
            rec = {}
            for base, typ, name, v in r.emissions_from(res, i):
                complete = name if not base else (base if not name else base + "." + name)
                key = typ + ":" + complete
                wild = typ + ":" + (base + ".*" if base else "*")
                val = {"l": v} if isinstance(v, int) else v
                for hit in (key in need, wild in need):
                    if hit:
                        rec.setdefault(key, []).append(val)
            assert rec == json.loads(r.record_json(i)), i


def test_crlf_terminators_gpu(oracle):
    """Hadoop LineRecordReader terminators: "\\r\\n", lone '\\r' and '\\n' end a
    line and are not part of it (ApacheHttpdLogfileRecordReader.java:57, 115)"""
    import corpora
    lines = lpa.synth_combined(20261019, 0, 20000).split(b"\n")[:-1]
    data = corpora.crlf_join(lines, 9)
    assert corpora.split_hadoop(data) == lines
    s, r = gpu_vs_oracle(oracle, "combined", paths(oracle), lines, allow_fallback=False, data=data)
    assert s["ok"] == 20000, s
    # terminator corners: counts and per-line status against the reference split
    rng = random.Random(4)
    pieces = [b"\r", b"\n", b"\r\n", b"\r\r", b"\n\r", b"\r\n\r\n", b"-", b"x", lines[0], lines[1]]
    o = oracle.Oracle("combined", paths(oracle))
    p = lpa.HttpdLoglineParser("combined", paths(oracle))
    for t in range(40):
        buf = b"".join(rng.choice(pieces) for _ in range(rng.randrange(1, 30)))
        want = corpora.split_hadoop(buf)
        r = p.parse_batch(buf)
        assert r.n_lines == len(want), (buf, r.n_lines, len(want))
        for i, l in enumerate(want):
            s1, r1 = o.parse_raw(l)
            assert int(r.status[i]) == s1, (buf, i, l)
            if s1 == oracle.OK:
                assert r.record_json(i) == r1


def test_utf8_text_gpu(oracle):
    """UTF-8 user agents and users stay on the device with exact records;
    UTF-8 in URIs, U+0085/U+2028/U+2029 and invalid sequences go to FALLBACK"""
    import corpora
    base = lpa.synth_combined(20261016, 0, 20000).split(b"\n")[:-1]
    s, _ = gpu_vs_oracle(oracle, "combined", paths(oracle), corpora.utf8_ua_lines(base, 5), allow_fallback=False)
    assert s["ok"] == 20000, s
    s, _ = gpu_vs_oracle(oracle, "combined", paths(oracle), corpora.utf8_hard_lines(base[:5000], 6))
    assert s["fallback"] > 1500 and s["ok"] > 900, s
    # both at once: UTF-8 user agents in a CRLF file
    lines = corpora.utf8_ua_lines(base, 8)
    s, _ = gpu_vs_oracle(oracle, "combined", paths(oracle), lines, allow_fallback=False,
                         data=corpora.crlf_join(lines, 10))
    assert s["ok"] == 20000, s


def expected_histograms(p, r, lines, oracle_fields_rec):
    """the lp_histograms words restated from the per-line results: statuses,
    the token columns of a host copy, and the records' status / method"""
    h = np.zeros(lpa.HIST_WORDS, dtype=np.int64)
    st = r.status
    h[0] = len(st)
    for s in (0, 1, 2):
        h[1 + s] = int((st == s).sum())
    buf, res = r.copy_to_host(with_input=False)
    cols = r.columns(res)
    ok = st == 0
    flags = cols[("tok_flags", 0)]
    k = 0
    while ("tok_span", k) in cols:
        sp = cols[("tok_span", k)].astype(np.int64)
        null = ok & (((flags >> k) & 1) == 1)
        h[16 + k] = int(null.sum())
        h[32 + k] = int((ok & ~null & ((sp >> 16) > (sp & 0xFFFF))).sum())
        k += 1
    for i in np.flatnonzero(ok):
        rec = oracle_fields_rec(i)
        s = rec.get("STRING:request.status.last", [None])[0]
        if s is not None and len(s) == 3 and s.isdigit() and 100 <= int(s) <= 599:
            h[100 + int(s)] += 1
        else:
            h[48] += 1
        m = rec.get("HTTP.METHOD:request.firstline.method", [None])[0]
        if m is None or m == "":
            h[64 + 16] += 1
        else:
            h[64 + (lpa.HIST_METHODS.index(m) if m in lpa.HIST_METHODS[:15] else 15)] += 1
    return h


def test_histograms_gpu(oracle):
    """lp_histograms (device run counters) against the same counts restated
    from the records and the token columns"""
    from test_emu_parity import mutate
    rng = random.Random(12)
    lines = lpa.synth_combined(20261020, 0, 6000).split(b"\n")[:-1]
    lines = [mutate(rng, l) if i % 3 == 0 else l for i, l in enumerate(lines)]
    for i in range(0, 6000, 97):  # other methods / status values
        lines[i] = lines[i].replace(b'"GET ', b'"PROPFIND ', 1).replace(b'" 200 ', b'" 999 ', 1)
    p = lpa.HttpdLoglineParser("combined", paths(oracle))
    r = p.parse_batch(b"".join(l + b"\n" for l in lines))
    got = np.array(p.histograms(), dtype=np.int64)
    want = expected_histograms(p, r, lines, lambda i: r.record(i))
    bad = np.flatnonzero(got != want)
    assert bad.size == 0, [(int(w), int(got[w]), int(want[w])) for w in bad[:20]]
    d = lpa.decode_histograms(got)
    assert d["lines"] == 6000 and d["bad"] > 100 and d["methods"].get("PROPFIND", 0) > 10
    assert sum(d["status"].values()) > 3000
    # into a device buffer (the RCCL all-reduce operand)
    import torch
    t = torch.zeros(lpa.HIST_WORDS, dtype=torch.int64, device="cuda")
    p.histograms(device_ptr=t.data_ptr())
    assert (t.cpu().numpy() == got).all()


def test_upstream_lists_and_binary_ip_gpu(oracle):
    from test_emu_parity import UPSTREAM_FMT, upstream_lines
    fields = oracle.possible_paths(UPSTREAM_FMT)
    s, _ = gpu_vs_oracle(oracle, UPSTREAM_FMT, fields, upstream_lines(20000, 5))
    assert s["ok"] > 10000, s


@pytest.mark.parametrize("which", [0, 1])
def test_request_cookies_gpu(oracle, which):
    from test_emu_parity import COOKIE_FMT, cookie_lines
    fields = [["HTTP.COOKIE:request.cookies.*"],
              ["HTTP.COOKIE:request.cookies.session", "HTTP.COOKIE:request.cookies.theme",
               "HTTP.COOKIES:request.cookies", "STRING:request.status.last"]][which]
    s, _ = gpu_vs_oracle(oracle, COOKIE_FMT, fields, cookie_lines(20000, 11 + which))
    # exactly the corpus's lines outside the device guard (7.6 % / 7.9 %: the
    # 5 % with an invalid escape "%zz" and the 3 % with a non-ASCII value the
    # generator plants; the same counts as the CPU emulation of the device code)
    assert s == [{"ok": 18476, "bad": 0, "fallback": 1524}, {"ok": 18414, "bad": 0, "fallback": 1586}][which], s


def test_querystring_token_gpu(oracle):
    from test_emu_parity import QS_FMT, querystring_lines
    s, _ = gpu_vs_oracle(oracle, QS_FMT, ["STRING:request.querystring.*"], querystring_lines(20000, 13))
    assert s == {"ok": 19177, "bad": 0, "fallback": 823}, s  # 4.1 %: the planted invalid escapes


def test_iso8601_timestamps_gpu(oracle):
    from test_emu_parity import ISO_FMT, iso_lines
    fields = oracle.possible_paths(ISO_FMT)
    s, _ = gpu_vs_oracle(oracle, ISO_FMT, fields, iso_lines(20000, 21), allow_fallback=False)
    assert s["ok"] > 12000 and s["bad"] > 1500, s


def test_upstream_cache_status_gpu(oracle):
    from test_emu_parity import CACHE_FMT, cache_status_lines
    fields = oracle.possible_paths(CACHE_FMT)
    s, _ = gpu_vs_oracle(oracle, CACHE_FMT, fields, cache_status_lines(20000, 9), allow_fallback=False)
    assert s["ok"] > 14000 and s["bad"] > 2000, s


@pytest.mark.parametrize("which", [0, 1])
def test_set_cookies_gpu(oracle, which):
    """ResponseSetCookieListDissector + ResponseSetCookieDissector on the
    device path (guard) and the replay, against the oracle"""
    from test_emu_parity import SETCOOKIE_FMT, SETCOOKIE_FIELDS, setcookie_lines
    s, _ = gpu_vs_oracle(oracle, SETCOOKIE_FMT, SETCOOKIE_FIELDS[which], setcookie_lines(20000, 31 + which))
    # The corpus plants inputs outside the restated subset (Max-Age / Version,
    # quotes, '$' / reserved names, names without '=', bad dates): 42.5 % /
    # 46.7 % FALLBACK.  With which=0 every FALLBACK line is one the oracle
    # refuses too (ORC_UNSUPPORTED: HttpCookie's RFC 2965 branch, parity
    # unpinned); with which=1, 391 lines (2.0 %) are FALLBACK on the device
    # only (an expires value outside the guard's `EEE, dd-MMM-yyyy HH:mm:ss
    # GMT` subset: other zones / layouts, or a ',' inside a value before it).
    assert s == [{"ok": 11503, "bad": 0, "fallback": 8497}, {"ok": 10659, "bad": 0, "fallback": 9341}][which], s


def test_setters_and_remapping_gpu():
    """parse(line, record) through setters (Parser.store rules, SetterPolicy,
    Long setters on STRING_OR_LONG paths, lp_casts) and a type remapping, on
    the engine"""
    import datetime
    from test_setters import Rec
    line = ('1.2.3.4 - - [10/Oct/2020:13:55:36 -0700] "GET /a?g=http%3A%2F%2Fx.y%2Fz&Q=1 HTTP/1.1" 200 - '
            '"http://ref.example:8080/x" "UA"')
    p = lpa.HttpdLoglineParser("combined")
    p.add_parse_target("TIME.EPOCH:request.receive.time.epoch", setter="set_long", value_class=int)
    p.add_parse_target("BYTESCLF:response.body.bytes", setter="set_long", value_class=int,
                       setter_policy=lpa.SetterPolicy.NOT_NULL)
    p.add_parse_target("STRING:request.firstline.uri.query.*", setter="set_string")
    p.add_parse_target("HTTP.PORT:request.referer.port", "TIME.MONTHNAME:request.receive.time.monthname",
                       setter="set_string")
    p.add_parse_target("HTTP.PORT:request.referer.port", setter="set_long", value_class=int)
    p.add_type_remapping("request.firstline.uri.query.g", "HTTP.URI")
    p.add_parse_target("HTTP.URI:request.firstline.uri.query.g", setter="set_string")
    assert p.get_casts("TIME.EPOCH:request.receive.time.epoch") == lpa.STRING_OR_LONG
    assert p.get_casts("STRING:request.firstline.uri.query.*") == lpa.STRING_ONLY
    assert p.get_casts("HTTP.URI:request.firstline.uri.query.g") == lpa.STRING_ONLY
    r = p.parse(line, Rec())
    epoch = int(datetime.datetime(2020, 10, 10, 13, 55, 36,
                                  tzinfo=datetime.timezone(datetime.timedelta(hours=-7))).timestamp()) * 1000
    assert r.l == {"TIME.EPOCH:request.receive.time.epoch": epoch, "HTTP.PORT:request.referer.port": 8080}
    assert r.s == {"STRING:request.firstline.uri.query.g": "http://x.y/z", "STRING:request.firstline.uri.query.q": "1",
                   "HTTP.URI:request.firstline.uri.query.g": "http://x.y/z",
                   "HTTP.PORT:request.referer.port": "8080",
                   "TIME.MONTHNAME:request.receive.time.monthname": "October"}
    # a Double setter on a STRING_OR_LONG path is never called: FatalErrorDuringCallOfSetterMethod
    q = lpa.HttpdLoglineParser("combined")
    q.add_parse_target("BYTES:response.body.bytes", setter="set_double", value_class=float)
    with pytest.raises(lpa.FatalErrorDuringCallOfSetterMethod):
        q.parse(line.replace(" 200 - ", " 200 512 "), Rec())


def test_result_table_gpu(demolog_lines):
    """lp_result_table (ParsedRecord / Hive SerDe columns) equals the records:
    per row the last non-null value of the path, converted as Value.getLong /
    getDouble; lines not OK have no values; a column type outside the path's
    casts is refused"""
    from logparser_amd.setters import Value
    fields = lpa.get_possible_paths("combined")
    data = b"".join(l + b"\n" for l in demolog_lines) + lpa.synth_combined(7, 0, 20000) + b"garbage line\n"
    p = lpa.HttpdLoglineParser("combined", fields)
    r = p.parse_batch(data)
    _, res = r.copy_to_host()
    cols = [("TIME.EPOCH:request.receive.time.epoch", int), ("BYTESCLF:response.body.bytes", int),
            ("HTTP.PATH:request.firstline.uri.path", str),
            ("STRING:request.firstline.uri.query.username", str), ("HTTP.HOST:request.referer.host", str),
            ("TIME.MONTHNAME:request.receive.time.monthname", str), ("HTTP.PORT:request.referer.port", int),
            ("STRING:request.status.last", str)]
    t = r.table_from(res, cols, threads=8)
    n_ok = 0
    for i in range(r.n_lines):
        rec = r.record(i) if r.status[i] == lpa.LINE_OK else {}
        n_ok += r.status[i] == lpa.LINE_OK
        for path, typ in cols:
            vals, ok = t[path]
            want = None
            for v in rec.get(path, []):
                v = v["l"] if isinstance(v, dict) else v
                if v is None:
                    continue
                x = Value(v)
                c = x.get_string() if typ is str else x.get_long() if typ is int else x.get_double()
                if c is not None:
                    want = c
            got = (vals[i] if ok[i] else None) if typ is str else (vals[i].item() if ok[i] else None)
            assert got == want, (i, path, got, want)
    assert n_ok > 20000
    # BYTESCLF is STRING_OR_LONG: a DOUBLE column finds no setter
    with pytest.raises(ValueError):
        r.table_from(res, [("BYTES:response.body.bytes", float)])


def test_strftime_conversions_gpu(oracle):
    """Every strftime conversion the reference converts (tests/strf_corpus.py:
    printed and mutated values of 13 patterns, the reference's MultiFields
    pattern among them) on the device against the oracle."""
    import strf_corpus
    tot = {"ok": 0, "bad": 0, "fallback": 0}
    for fmt, lines in strf_corpus.corpus(20261017, per_pattern=400):
        s, _ = gpu_vs_oracle(oracle, fmt, strf_corpus.FIELDS, lines)
        for k in tot:
            tot[k] += s[k]
        assert s["fallback"] <= len(lines) // 10, (fmt, s)
    print("strftime corpus on the device:", tot)
    assert tot["ok"] > 3000 and tot["bad"] > 500, tot


def test_type_remapping_gpu(oracle):
    """Parser.addTypeRemapping (core/Parser.java:636-677): query parameters
    holding URLs (and a user agent) remapped to HTTP.URI and dissected again
    on the device -- derived URI stages (k_derived_lines) on values in the
    input and decoded values in the arena, a remapped parameter of a remapped
    URL, a remapping to a type without dissectors; exact against the oracle."""
    import remap_corpus as rc
    lines = rc.corpus(11, 6000)
    s, r = gpu_vs_oracle(oracle, rc.FORMAT, rc.FIELDS, lines, remaps=rc.REMAPS)
    print("type remapping corpus:", s)
    assert s["ok"] > 3000, s
    assert s["fallback"] < 0.4 * len(lines), s


def _device_vs_host_table(r, res, columns):
    """lp_result_table built on the GPU (device view) equals the host table
    (the replay) column by column: validity, values, Arrow offsets and bytes.
    Returns the paths whose values only the host derives (FallbackRequired)."""
    host_only = []
    chunks = []  # calls of at most 24 columns with distinct paths (the results are keyed by path)
    for c in columns:
        for ch in chunks:
            if len(ch) < 24 and all(x[0] != c[0] for x in ch):
                ch.append(c)
                break
        else:
            chunks.append([c])
    for chunk in chunks:
        dev_cols = []
        for c in chunk:
            try:
                r.table_device([c])
                dev_cols.append(c)
            except lpa.FallbackRequired:
                host_only.append(c[0])
        if not dev_cols:
            continue
        h = r.table_from(res, dev_cols, threads=8, decode=False)
        d = r.table_device(dev_cols)
        for path, typ in dev_cols:
            hv, hok = h[path]
            dv, dok = d[path]
            dok = dok.cpu().numpy().astype(bool)
            assert (hok == dok).all(), (path, int(np.argmax(hok != dok)))
            if typ is str:
                (hoff, hchars), (doff, dchars) = hv, dv
                doff = doff.cpu().numpy()
                assert (hoff == doff).all(), (path, int(np.argmax(hoff != doff)))
                assert hchars[:hoff[-1]].tobytes() == dchars.cpu().numpy().tobytes(), path
            else:
                dv = dv.cpu().numpy()
                assert (hv[hok] == dv[hok]).all(), path
    return host_only


def test_device_table_gpu(demolog_lines):
    """lp_result_table on the device (the Hive / ParsedRecord columns built in
    HBM) equals the host table on every path of 'combined' as STRING and LONG
    (casts permitting) columns, on the demo log,
    synthetic config-2 lines and a garbage line"""
    fields = lpa.get_possible_paths("combined")
    data = b"".join(l + b"\n" for l in demolog_lines) + lpa.synth_combined(7, 0, 30000) + b"garbage line\n"
    p = lpa.HttpdLoglineParser("combined", fields)
    r = p.parse_batch(data)
    _, res = r.copy_to_host()
    cols = []
    for f in fields:
        if f.endswith("*"):
            continue
        cols.append((f, str))
        casts = p.get_casts(f) or 0
        if casts & lpa.CAST_LONG:
            cols.append((f, int))
    cols += [("STRING:request.firstline.uri.query.username", str), ("STRING:request.firstline.uri.query.q", str)]
    # DOUBLE columns (casts permitting): a long-valued source is built on the device; Double.parseDouble
    # of a string-valued token stays with the host table (FallbackRequired)
    dbl = [f for f in fields if not f.endswith("*") and (p.get_casts(f) or 0) & lpa.CAST_DOUBLE]
    cols += [(f, float) for f in dbl]
    host_only = _device_vs_host_table(r, res, cols)
    assert set(host_only) <= set(dbl), host_only
    # the timed batch size: a whole config-2 batch in one call
    big = lpa.synth_combined(11, 0, 2_000_000)
    r2 = p.parse_batch(big)
    t = r2.table_device([("IP:connection.client.host", str), ("TIME.EPOCH:request.receive.time.epoch", int),
                         ("HTTP.PATH:request.firstline.uri.path", str)])
    assert int(t["TIME.EPOCH:request.receive.time.epoch"][1].sum()) == r2.counters["ok"]


def test_device_table_other_configs_gpu():
    """The device table on configs 3 (strftime), 4 (NGINX upstream: its list
    items and converted times from the URI kernel's item tables and phase 1's
    millisecond columns) and 5 (three LogFormats, rows of formats without a
    path empty), and on type-remapped paths"""
    import remap_corpus as rc
    from test_emu_parity import (COOKIE_FMT, QS_FMT, UPSTREAM_FMT, SETCOOKIE_FMT, SETCOOKIE_FIELDS, cookie_lines,
                                 querystring_lines, upstream_lines, setcookie_lines)
    cases = [(wl, lpa.SYNTH_FORMATS[wl], lpa.synth(wl, 5, 0, 20000), ()) for wl in (3, 4, 5)]
    # request cookies, raw-token query strings and Set-Cookie lists (the URI kernel's pair stages;
    # ResponseSetCookieDissector's outputs from the device table), upstream address / status lists
    # and the binary IP (its list stages, phase 1's BinaryIP stage)
    extra = {COOKIE_FMT: ["HTTP.COOKIE:request.cookies.session", "HTTP.COOKIE:request.cookies.theme"],
             QS_FMT: ["STRING:request.querystring.aap", "STRING:request.querystring.res"],
             SETCOOKIE_FMT: [f for f in SETCOOKIE_FIELDS[1] if f.startswith(("HTTP.SETCOOKIE:", "STRING:response",
                                                                            "TIME.EPOCH:"))] +
             ["HTTP.SETCOOKIE:response.cookies.session", "STRING:response.cookies.session.path",
              "TIME.EPOCH:response.cookies.session.expires", "STRING:response.cookies.nba-1.expires",
              "HTTP.SETCOOKIE:response.cookies.x.y", "STRING:response.cookies.x.y.value",
              "STRING:response.cookies.x.y.domain", "STRING:response.cookies._ga.comment"]}
    for fmt, lines in ((COOKIE_FMT, cookie_lines(5000, 21)), (QS_FMT, querystring_lines(5000, 22)),
                       (UPSTREAM_FMT, upstream_lines(5000, 23)), (SETCOOKIE_FMT, setcookie_lines(5000, 32))):
        cases.append((6, fmt, b"".join(l + b"\n" for l in lines), ()))
    rlines = rc.corpus(3, 3000)
    cases.append((0, rc.FORMAT, b"".join(l + b"\n" for l in rlines), rc.REMAPS))
    for wl, fmt, data, remaps in cases:
        fields = [f for f in lpa.get_possible_paths(fmt) if not f.endswith("*")] if not remaps else rc.FIELDS
        fields = fields + extra.get(fmt, [])
        p = lpa.HttpdLoglineParser(fmt, fields)
        for n, t in remaps:
            p.add_type_remapping(n, t)
        r = p.parse_batch(data)
        _, res = r.copy_to_host()
        cols = [(f, str) for f in fields if not f.endswith("*")]
        cols += [(f, int) for f in fields if not f.endswith("*") and (p.get_casts(f) or 0) & lpa.CAST_LONG]
        cols += [(f, float) for f in fields if not f.endswith("*") and (p.get_casts(f) or 0) & lpa.CAST_DOUBLE]
        host_only = _device_vs_host_table(r, res, cols)
        print(fmt[:40], "host-only columns:", host_only)
        if remaps:
            # the remapped deliveries themselves, and the outputs under "url.query.next": a base query
            # parameter literally named "url.query.next" would be remapped too (the remapping is by
            # name), so two stages deliver there and the host table keeps their order
            assert all(h in ("HTTP.URI:" + rc.REMAPS[0][0], "SOMETAG:request.firstline.uri.query.tag") or
                       ".url.query.next." in h for h in host_only), host_only
        else:  # every path of configs 3-5 and of the cookie / query-string / upstream corpora from device
            # columns (list items, SECOND_MILLIS -> MILLISECONDS -> MICROSECONDS, binary IPs, cookies, raw
            # query parameters included)
            assert host_only == [], host_only


@pytest.mark.gpu
@pytest.mark.parametrize("wl", [3, 4])
def test_chunk_excess_instances_gpu(oracle, wl):
    """Chunks of more than 64 lines (chunk_excess: their 65th line on queued
    for k_parse_ovf_lines) and lines that need the backtracking DFS (queued
    too: the chunk kernel has no DFS) on the kernel instances other than the
    Apache common / combined one: config 3's strftime program and config 4's
    literal-aware NGINX program, against the oracle line by line.  Regression
    for the round-5 fault: chunk_excess numbered fewer lines than the staging
    pass (wrong lane ids in the non-inlined call), leaving
    line_off entries unwritten; the kernels' self-check (Meta::err) now fails
    such a batch instead of faulting."""
    rng = random.Random(11 + wl)
    fmt = lpa.SYNTH_FORMATS[wl]
    base = lpa.synth(wl, 20261022, 0, 4000).split(b"\n")[:-1]
    lines = []
    for i, l in enumerate(base):
        lines.append(l)
        if i % 400 == 5:
            lines += [b"x"] * rng.randrange(70, 260)  # > 64 line starts in one chunk
        if i % 300 == 17:
            lines.append(b"-" * rng.randrange(1, 5))  # short lines between them
    fields = paths(oracle, fmt)
    s, r = gpu_vs_oracle(oracle, fmt, fields, lines)
    assert s["ok"] > 3500, s
    assert r.diag["overflow_waves"] > 1000, r.diag  # (chunked: lines queued for k_parse_ovf_lines)


@pytest.mark.gpu
def test_chunk_geometry_gpu(oracle):
    """The one-pass parse kernel's byte chunks (LP_OPT_CHUNK_LINES): the same
    results whatever the chunk size -- chunks of a few lines, chunks holding
    more than 64 lines (runs of very short lines: chunk_excess and
    k_parse_ovf_lines), lines longer than a chunk's window, CRLF / lone-CR
    terminators and a last line without one.  The default geometry is
    checked line by line against the oracle, every other one against it."""
    import corpora
    rng = random.Random(7)
    base = lpa.synth_combined(20261020, 0, 6000).split(b"\n")[:-1]
    lines = []
    for i, l in enumerate(base):
        lines.append(l)
        if i % 500 == 7:
            lines += [b"x"] * rng.randrange(100, 300)  # > 64 line starts in one chunk
        if i % 700 == 11:
            lines.append(l[:-1] + b"a" * rng.randrange(3000, 7000) + b'"')  # longer than a window
    data = corpora.crlf_join(lines, 5)  # the last line unterminated
    want = corpora.split_hadoop(data)
    assert want == lines
    fields = paths(oracle)
    s, r0 = gpu_vs_oracle(oracle, "combined", fields, lines, data=data)
    assert s["ok"] > 5900, s
    recs0 = [r0.record_json(i) if int(r0.status[i]) == lpa.LINE_OK else None for i in range(len(lines))]
    for cl in (1, 17, 64):
        p = lpa.HttpdLoglineParser("combined", fields, options={lpa.OPT_CHUNK_LINES: cl})
        r = p.parse_batch(data)
        assert r.n_lines == len(lines), (cl, r.n_lines, len(lines))
        assert (r.status == r0.status).all(), (cl, int(np.argmax(r.status != r0.status)))
        for i in range(len(lines)):
            if recs0[i] is not None:
                assert r.record_json(i) == recs0[i], (cl, i)
        assert r.counters == r0.counters, cl
    # every chunk whose line number is not known at its first poll goes to the
    # deferred pass (LP_OPT_CHUNK_WAIT < 0): the same results; on a larger
    # batch too (many chunks deferred, a deferred pass over many waves)
    big = lpa.synth_combined(20261021, 0, 300000)
    pb = lpa.HttpdLoglineParser("combined", fields)
    rb0 = pb.parse_batch(big)
    assert rb0.diag["deferred_chunks"] == 0
    # -2: the odd chunks deferred, the even ones finished by k_parse_chunks
    # (line_off boundaries between a finished and a deferred chunk; the last
    # chunk's sentinel from either pass), and a small positive wait
    n_chunks = {}  # (-1 defers every chunk: their number)
    for d, wait in ((data, -1), (big, -1), (data, -2), (big, -2), (big, 8)):
        ref = r0 if d is data else rb0
        p = lpa.HttpdLoglineParser("combined", fields, options={lpa.OPT_CHUNK_WAIT: wait})
        r = p.parse_batch(d)
        nd = r.diag["deferred_chunks"]
        if wait == -1:
            assert nd > 1, r.diag
            n_chunks[id(d)] = nd
        elif wait == -2:
            assert 0 < nd <= n_chunks[id(d)] // 2 + 1, (nd, n_chunks[id(d)])  # the odd ones
        else:
            assert 0 <= nd <= n_chunks[id(d)], r.diag
        assert r.n_lines == ref.n_lines and (r.status == ref.status).all()
        assert r.counters == ref.counters
        for i in range(0, ref.n_lines, 1 if d is data else 37):
            if int(ref.status[i]) == lpa.LINE_OK:
                assert r.record_json(i) == ref.record_json(i), i
