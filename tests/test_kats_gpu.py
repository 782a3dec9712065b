"""The reference's own known-answer tests, through libpsx on the GPU.

store_test.cpp's EXPECT_EQ values (tests/golden/reference_kats.json) are fed to the HIP
path as serialized sparse records — one {row 0, n = 1, col, delta} record per Inc, in the
test's order — and the reference's expected values are asserted directly on the rows
the device holds (dense: VectorStore; sorted-map: SortedVectorMapStore; the same Incs on
a MapStore row must give the same values).  Each case runs twice: every record in one
message (the ordered path's > 64-records-per-row walk for SShrink), and the records
spread over fused calls of up to 16 messages.
"""
import json
import os

import numpy as np
import pytest

torch = pytest.importorskip("torch")

import parameter_server_amd as psa
from parameter_server_amd import wire

pytestmark = pytest.mark.gpu

GOLDEN = os.path.join(os.path.dirname(__file__), "golden")
KATS = json.load(open(os.path.join(GOLDEN, "reference_kats.json")))
SURVEY = json.load(open(os.path.join(GOLDEN, "survey_recorded.json")))


@pytest.fixture(scope="module", autouse=True)
def _gpu(built_lib):
    if not torch.cuda.is_available():
        pytest.skip("no GPU")


def _server(kind, cap, nsenders):
    srv = psa.Server(0, 1, list(range(100, 100 + nsenders)))
    max_entries = 512 if kind != psa.ROW_DENSE else 0
    srv.CreateTable(0, psa.TableInfo(row_kind=kind, dtype=psa.I32, row_capacity=max(cap, 1),
                                     oplog_dense_serialized=False, max_rows=1, max_entries=max_entries))
    if kind == psa.ROW_DENSE:   # VectorStore::Init(capacity) zeroes the row (vector_store.hpp:64-67)
        srv.load_rows(0, 0, np.zeros((1, cap), np.int32))
    return srv


def _records(ops):
    return [(0, np.array([c], np.int32), np.array([d], np.int32)) for c, d in ops]


def _run(srv, ops, split):
    """split: None = all ops in one message; else ops per message (fused 16 per call)."""
    if not ops:
        return
    if split is None:
        msgs = [wire.sparse_stream_np(0, 4, _records(ops))]
    else:
        msgs = [wire.sparse_stream_np(0, 4, _records(ops[i:i + split])) for i in range(0, len(ops), split)]
    dev = [torch.from_numpy(np.array(m, copy=True)).cuda() for m in msgs]
    torch.cuda.synchronize()
    ver = {}
    for k in range(0, len(dev), 16):
        call = []
        for j, d in enumerate(dev[k:k + 16]):
            bg = 100 + j
            ver[bg] = ver.get(bg, -1) + 1
            call.append((d.data_ptr(), d.numel(), bg, ver[bg]))
        srv.apply_device(call)
    srv.sync()


def _get_map(srv, kind):
    """{col: value} of row 0 as the device serializes it (ServerRow::Serialize)."""
    raw = srv.serialize_rows(0, [0])
    if not raw:
        return {}
    body = np.frombuffer(raw[12:], np.int32).reshape(-1, 2)
    return {int(c): int(v) for c, v in body}


def _entries_in_order(srv):
    raw = srv.serialize_rows(0, [0])
    return np.frombuffer(raw[12:], np.int32).reshape(-1, 2).tolist() if raw else []


@pytest.mark.parametrize("split", [None, 1, 7], ids=["one_msg", "one_op_per_msg", "7_ops_per_msg"])
@pytest.mark.parametrize("name", sorted(KATS))
def test_store_test_kat_through_hip(name, split):
    case = KATS[name]
    dense = case["store"].startswith("VectorStore")
    kinds = [psa.ROW_DENSE, psa.ROW_MAP] if dense else [psa.ROW_SORTED_MAP, psa.ROW_MAP]
    for kind in kinds:
        srv = _server(kind, case["init_capacity"], 16)
        _run(srv, case["ops"], split)
        if kind == psa.ROW_DENSE:
            row = srv.read_rows(0, 0, 1)[0]
            for col, want in case["expect"]:
                assert int(row[col]) == want, (name, col)
            if "expect_capacity" in case:
                assert row.size == case["expect_capacity"]
        else:
            m = _get_map(srv, kind)
            for col, want in case["expect"]:        # Get() of an absent key is 0
                assert m.get(col, 0) == want, (name, kind, col)
            assert 0 not in m.values()               # zeros are removed (Inc: Remove on 0)
        srv.close()


def test_row_test_recorded_order_through_hip():
    """row_test.cpp's Inc sequence on a SortedVectorMapRow<int32> (cross-check against the
    order SURVEY.md §4 recorded from running it; row_test asserts nothing itself)."""
    case = SURVEY["RowTestSortedVectorMapRow"]
    srv = _server(psa.ROW_SORTED_MAP, 0, 16)
    _run(srv, case["ops"], None)
    assert _entries_in_order(srv) == case["expect_entries_in_order"]
    assert len(srv.serialize_rows(0, [0])) - 12 == case["expect_serialized_bytes"]
