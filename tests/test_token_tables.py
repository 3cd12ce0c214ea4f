"""The planner's (plan.cpp) and the oracle's (oracle.c) token tables against
the tables extracted from the reference's Java sources by
tests/golden/extract_token_tables.py (committed as tests/golden/token_tables.json).

plan.cpp and oracle.c are two hand transcriptions of
ApacheHttpdLogFormatDissector.createAllTokenParsers (:199-638) and the
nginxmodules/*Module.getTokenParsers tables; checking each against a
mechanical extraction removes the risk of both sharing one transcription
error (token, regex, priority, output type/name/casts, order)."""
import json
import os

import pytest

import emu_lib
import oracle_lib

HERE = os.path.dirname(os.path.abspath(__file__))
GOLDEN = os.path.join(HERE, "golden", "token_tables.json")
REFERENCE = "/root/reference"


def golden():
    with open(GOLDEN, encoding="utf-8") as f:
        return json.load(f)


def diff(got, want):
    problems = []
    if len(got) != len(want):
        problems.append("length %d != %d" % (len(got), len(want)))
    for i, (g, w) in enumerate(zip(got, want)):
        if g != w:
            problems.append("#%d got %r\n     want %r" % (i, g, w))
    return problems


@pytest.mark.parametrize("family", ["apache", "nginx"])
def test_planner_table_matches_reference(family):
    got = emu_lib.token_table(family == "nginx")
    assert diff(got, golden()[family]) == []


@pytest.mark.parametrize("family", ["apache", "nginx"])
def test_oracle_table_matches_reference(family):
    got = oracle_lib.token_table(family == "nginx")
    assert diff(got, golden()[family]) == []


def test_golden_tables_shape():
    g = golden()
    # the whole Apache table: %%, 57 first/last triples, 7 named, 3 strftime
    kinds = [p["kind"] for p in g["apache"]]
    assert (kinds.count("fixed"), kinds.count("plain"), kinds.count("named"), kinds.count("param")) == (1, 171, 7, 3)
    assert g["fl_original_tokens"] == ["%s", "%U", "%T", "%{us}T", "%{ms}T", "%{s}T", "%D", "%r"]
    assert g["nginx_modules"][:2] == ["CoreLogModule", "UpstreamModule"]
    toks = {p["token"] for p in g["nginx"]}
    for t in ("$remote_addr", "$upstream_addr", "$ssl_protocol", "$geoip_city", "$namespace"):
        assert t in toks


@pytest.mark.skipif(not os.path.isdir(REFERENCE), reason="reference sources not present")
def test_golden_tables_regenerate_identically(tmp_path):
    """the committed JSON is what the extractor derives from the reference now"""
    import importlib.util
    spec = importlib.util.spec_from_file_location("extract_token_tables",
                                                  os.path.join(HERE, "golden", "extract_token_tables.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    assert mod.extract(REFERENCE) == golden()
