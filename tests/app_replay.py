"""Replay of an App-API driver's trace (libpetuum_ps.so with PSX_TRACE_DIR: every
ClientSendOpLogMsg handed to a shard, every row request and reply, every push body)
through one oracle ServerThread per shard — test infrastructure only.  Every reply and
every push body the GPU shards produced must be byte-identical to the oracle's."""
import struct

import numpy as np

from parameter_server_amd import wire, ServerThread
from oracle_backend import OracleBackend


def replay(trace, channels, tables, client_id=0):
    """tables: dicts {tid, kind, dtype, cap, dense_serialized[, version_maintain, adarevision]}
    in creation order.  Returns the event counts."""
    events = [ln.split() for ln in open(trace / "index.txt").read().splitlines()]
    threads, got_push, want_push, got_reply, want_reply = [], [], [], [], []
    for ch in range(channels):
        bg = client_id * 1000 + 100 + ch
        be = OracleBackend([bg], num_clients=1)
        for t in tables:
            be.create(t["tid"], t["kind"], t["dtype"], t["cap"], dense_serialized=t.get("dense_serialized", True),
                      version_maintain=t.get("version_maintain", False), adarevision=t.get("adarevision"))
        want_push.append([])
        want_reply.append([])
        got_push.append([])
        got_reply.append([])
        threads.append(ServerThread(
            be, push=lambda bodies, clock, ch=ch: want_push[ch].append(bodies[0]),
            reply=lambda bg_, t_, r_, clock, rec, ch=ch: want_reply[ch].append(rec)))
    counts = {"msg": 0, "push": 0, "req": 0, "reply": 0, "clock_msg": 0}
    for kind, ch, seq, name in events:
        ch = int(ch)
        bg = client_id * 1000 + 100 + ch
        data = (trace / name).read_bytes()
        counts[kind] += 1
        if kind == "msg":
            h, payload = wire.decode_oplog_msg(np.frombuffer(data, np.uint8))
            assert h["client_id"] == client_id
            counts["clock_msg"] += 1 if h["is_clock"] else 0
            threads[ch].HandleOpLogMsg(bg, payload, bool(h["is_clock"]), h["bg_clock"], h["version"])
        elif kind == "req":
            tid, row = struct.unpack("<ii", data)
            assert threads[ch].HandleRowRequest(bg, tid, row, 0)
        elif kind == "reply":
            got_reply[ch].append(data)
        else:
            got_push[ch].append(data)
    for ch in range(channels):
        assert len(got_reply[ch]) == len(want_reply[ch])
        for i, (g, w) in enumerate(zip(got_reply[ch], want_reply[ch])):
            assert g == w, f"shard {ch} reply {i} differs"
        assert len(got_push[ch]) == len(want_push[ch]), (len(got_push[ch]), len(want_push[ch]))
        for i, (g, w) in enumerate(zip(got_push[ch], want_push[ch])):
            assert g == w, f"shard {ch} push {i} differs"
    return counts
