"""Shared helpers to check a parsed canonical record against the transcribed
reference vectors in tests/golden/reference_vectors.json."""
import json
import os

HERE = os.path.dirname(os.path.abspath(__file__))
VECTORS = os.path.join(HERE, "golden", "reference_vectors.json")


def load_vectors():
    with open(VECTORS, encoding="utf-8") as f:
        return json.load(f)


def check_case(case, status, record):
    """status: 0 OK / 1 BAD.  record: canonical dict path -> [values]."""
    problems = []
    if case["bad"]:
        if status != 1:
            problems.append("expected DissectionFailure, got status %s" % status)
        return problems
    if status != 0:
        return ["expected OK, got status %s" % status]
    for path, want in case["expect"].items():
        got = record.get(path)
        if got is None:
            # Map-based reference records read "null" for an absent field
            # too; DissectorTester cases mean "present AND null"
            if want is None and not case.get("null_present"):
                continue
            problems.append("%s: absent, want %r" % (path, want))
        elif want not in got:
            problems.append("%s: got %r, want %r" % (path, got, want))
    for path in case["absent"]:
        if path in record:
            problems.append("%s: present %r, want absent" % (path, record[path]))
    return problems
