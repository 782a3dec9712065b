"""bench.c5_schedule — the SSP arrival order C5 is measured on: workers of
different speeds, Get gated at staleness 4 (ssp_push_consistency_controller.cpp:70-88), the
server's min clock and pushes (server.cpp:62-79, server_thread.cpp:262-288)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402


def test_gate_and_push_order():
    B, clocks, s = 8, 20, 4
    arr, st = bench.c5_schedule(B, clocks, staleness=s)
    assert len(arr) == B * clocks
    seen = [0] * B
    pushed, push_at = 0, {0: -1}
    for i, (w, c, push) in enumerate(arr):
        assert c == seen[w]                    # each worker's clocks arrive in order
        seen[w] += 1
        # the worker started clock c only once clock c - s had been pushed
        need = c - s
        if need > 0:
            assert need in push_at and push_at[need] < i, (w, c)
        if push:
            assert push == pushed + 1 and push == min(seen)
            pushed = push
            push_at[push] = i
    assert pushed == clocks
    assert st["max_clock_lead"] == s + 1     # the fastest worker is held at the gate
    assert st["gate_blocks"] > 0


def test_equal_speeds_need_no_gate():
    arr, st = bench.c5_schedule(4, 10, speeds=[1.0] * 4)
    assert st["gate_blocks"] == 0 and st["max_clock_lead"] <= 1
    assert [p for _, _, p in arr if p] == list(range(1, 11))
