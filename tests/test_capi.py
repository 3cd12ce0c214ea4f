"""CPU-side checks of the product C ABI: the in-tree library loads, exports
every entry point include/logparser_amd.h declares, answers setup-time
questions, and refuses to run without a GPU (no CPU fallback)."""
import ctypes
import os
import re

import pytest

import logparser_amd as lpa

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def declared_symbols():
    with open(os.path.join(ROOT, "include", "logparser_amd.h")) as f:
        src = f.read()
    return sorted(set(re.findall(r"\b(lp_[a-z_]+)\s*\(", src)))


def test_library_exports_every_declared_symbol():
    L = ctypes.CDLL(lpa.LIB_PATH)
    syms = declared_symbols()
    assert len(syms) >= 14
    for s in syms:
        assert hasattr(L, s), s


def test_possible_paths_match_oracle(oracle):
    for fmt in ["combined", "common", "combinedio", "%h %{Cookie}i %{%Y-%m-%dT%H:%M:%S%z}t %q"]:
        assert lpa.get_possible_paths(fmt) == oracle.possible_paths(fmt), fmt


def test_synth_deterministic():
    a = lpa.synth_combined(7, 1000, 50)
    b = lpa.synth_combined(7, 1000, 50)
    c = lpa.synth_combined(7, 1025, 25)
    assert a == b
    assert a.split(b"\n")[25:] == c.split(b"\n")
    assert a.count(b"\n") == 50


def test_compile_requires_gpu():
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    p = lpa.HttpdLoglineParser("combined", ["IP:connection.client.host"])
    with pytest.raises(lpa.EngineUnavailable):
        p.parse_batch(b"1.2.3.4 - - [31/Dec/2012:23:00:44 -0700] \"GET / HTTP/1.1\" 200 1 \"-\" \"x\"\n")


def test_possible_paths_with_remapping():
    """Parser.getPossiblePaths with a type remapping (core/Parser.java:954-962):
    the remapped path and what the new type's dissectors produce below it."""
    base = set(lpa.get_possible_paths("combined"))
    got = set(lpa.get_possible_paths("combined", remaps=[("request.firstline.uri.query.g", "HTTP.URI", 1)]))
    assert base < got
    for p in ["HTTP.URI:request.firstline.uri.query.g", "HTTP.HOST:request.firstline.uri.query.g.host",
              "HTTP.QUERYSTRING:request.firstline.uri.query.g.query",
              "STRING:request.firstline.uri.query.g.query.*"]:
        assert p in got, p
    assert not any("query.g" in p for p in base)
