"""Pins the CPU oracle against the reference's own known-answer tests
(tests/golden/reference_kats.json: the EXPECT_EQ values of store_test.cpp), and
cross-checks it against SURVEY.md §4's recorded run of row_test.cpp
(tests/golden/survey_recorded.json; that test asserts nothing, so it pins nothing)."""
import json
import os

import numpy as np
import pytest

from oracle.oracle import OracleServer, DENSE, SORTED_MAP, MAP, I32

GOLDEN = os.path.join(os.path.dirname(__file__), "golden")
KATS = json.load(open(os.path.join(GOLDEN, "reference_kats.json")))
SURVEY = json.load(open(os.path.join(GOLDEN, "survey_recorded.json")))


def _server_for(case):
    kind = DENSE if case["store"].startswith("VectorStore") else SORTED_MAP
    s = OracleServer()
    s.create_table(0, kind, I32, case["init_capacity"], oplog_dense_serialized=False)
    if kind == DENSE:   # VectorStore::Init(capacity) zeroes the row (vector_store.hpp:64-67)
        s.load_dense_rows(0, 0, np.zeros((1, case["init_capacity"]), dtype=np.int32))
    return s


@pytest.mark.parametrize("name", sorted(KATS) + sorted(SURVEY))
def test_reference_kat(oracle_lib, name):
    case = KATS.get(name) or SURVEY[name]
    s = _server_for(case)
    for col, delta in case["ops"]:
        s.row_inc(0, 0, col, delta)
    for col, want in case["expect"]:
        assert s.get(0, 0, col) == want, (name, col)
    if "expect_entries_in_order" in case:
        raw = s.serialize_row(0, 0)
        assert len(raw) == case["expect_serialized_bytes"]
        ent = np.frombuffer(raw, dtype=np.int32).reshape(-1, 2).tolist()
        assert ent == case["expect_entries_in_order"]
    if "expect_capacity" in case:
        assert len(s.serialize_row(0, 0)) == 4 * case["expect_capacity"]


def test_sorted_map_store_order_invariants(oracle_lib):
    """SortedVectorMapStore keeps insertion-sorted order: new keys bubble backward past
    strictly smaller values (sorted_vector_map_store.hpp:264-285); adds to existing keys
    do not move them (:325-327); zeros are removed (:329-334)."""
    s = OracleServer()
    s.create_table(0, SORTED_MAP, I32, 0, oplog_dense_serialized=False)
    for col, d in [(5, 1), (6, 3), (7, 2), (5, 10), (8, 3), (6, -3)]:
        s.row_inc(0, 0, col, d)
    ent = np.frombuffer(s.serialize_row(0, 0), dtype=np.int32).reshape(-1, 2).tolist()
    # [(5,1)] -> [(6,3),(5,1)] -> [(6,3),(7,2),(5,1)] -> (5,11) in place
    # -> (8,3) appended, 3 > 11 is false so it stays last -> (6,0) removed.
    assert ent == [[7, 2], [5, 11], [8, 3]]


def test_map_store_erases_zero(oracle_lib):
    """MapStore::Inc erases an entry that reaches zero (map_store.hpp:60-65)."""
    s = OracleServer()
    s.create_table(0, MAP, I32, 0, oplog_dense_serialized=False)
    s.row_inc(0, 0, 3, 4)
    s.row_inc(0, 0, 9, 1)
    s.row_inc(0, 0, 3, -4)
    raw = s.serialize_row(0, 0)
    assert np.frombuffer(raw, dtype=np.int32).reshape(-1, 2).tolist() == [[9, 1]]
