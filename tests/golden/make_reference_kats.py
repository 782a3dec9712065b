"""Writes tests/golden/reference_kats.json: the known-answer vectors held by the
reference's own tests for the row stores on the apply path.

Each case is data transcribed from the reference test source (inputs and the
expected values its EXPECT_EQ lines state); no reference code is copied or run.
  store_test.cpp = tests/petuum_ps/storage/store_test.cpp
  row_test.cpp   = apps/lda/src/row_test.cpp

row_test.cpp holds inputs only (it LOGs its output and asserts nothing), so it is NOT a
reference-held vector: its inputs and the entry order SURVEY.md §4 recorded from running
it go to survey_recorded.json, a cross-check with that provenance, separate from the
reference's EXPECT_EQ values in reference_kats.json.
Run:  python tests/golden/make_reference_kats.py
"""
import json
import os

HERE = os.path.dirname(os.path.abspath(__file__))

kats = {
    "VectorInit": {   # store_test.cpp:34-37
        "store": "VectorStore<int>", "init_capacity": 100, "ops": [],
        "expect_capacity": 100, "expect": [],
    },
    "VectorGet": {    # store_test.cpp:39-41
        "store": "VectorStore<int>", "init_capacity": 100, "ops": [],
        "expect": [[5, 0]],
    },
    "VectorInc": {    # store_test.cpp:42-49
        "store": "VectorStore<int>", "init_capacity": 100,
        "ops": [[1, 5], [2, 10], [1, -2]],
        "expect": [[1, 3], [2, 10]],
    },
    "SGet": {         # store_test.cpp:76-78
        "store": "SortedVectorMapStore<int>", "init_capacity": 0, "ops": [],
        "expect": [[100, 0]],
    },
    "SIncGet": {      # store_test.cpp:80-92
        "store": "SortedVectorMapStore<int>", "init_capacity": 0,
        "ops": [[1, 2], [2, 0], [3, -9], [15, 8], [3, 12]],
        "expect": [[1, 2], [2, 0], [3, 3], [4, 0], [15, 8]],
    },
    "SShrink": {      # store_test.cpp:94-116
        "store": "SortedVectorMapStore<int>", "init_capacity": 0,
        "ops": [[i, i % 17] for i in range(300)] + [[i, -(i % 17)] for i in range(150, -1, -1)],
        # EXPECT_EQ(Get(i), 0) for i in [0,150]; the test's second loop (151..150) is
        # empty, so entries 151..299 are not asserted by the reference.
        "expect": [[i, 0] for i in range(151)],
    },
}

# Not reference-held (row_test.cpp asserts nothing): SURVEY.md §4's recorded run.
survey_recorded = {
    "RowTestSortedVectorMapRow": {   # row_test.cpp:11-46 (SortedVectorMapRow<int32_t>, Init(0))
        "store": "SortedVectorMapRow<int32_t>", "init_capacity": 0,
        "ops": [[1, 10], [13, 2], [112, 2], [22, 2], [13, 2], [1, -10]],
        "expect": [[13, 4], [112, 2], [22, 2], [1, 0]],
        # CopyToVector / Serialize order recorded by SURVEY.md §4 from the reference run.
        "expect_entries_in_order": [[13, 4], [112, 2], [22, 2]],
        "expect_serialized_bytes": 24,
    },
}

if __name__ == "__main__":
    with open(os.path.join(HERE, "reference_kats.json"), "w") as f:
        json.dump(kats, f, separators=(",", ":"))
    with open(os.path.join(HERE, "survey_recorded.json"), "w") as f:
        json.dump(survey_recorded, f, separators=(",", ":"))
    print("wrote", len(kats), "cases")
