"""BASELINE.json configurations at their full shapes on the GPU.

C2: the headline workload exactly as bench.py times it (2^20 rows x 256 f32, 8 full-coverage
messages in per-message random row order), bit-exact against the in-order fp32 sum
table + u_0 + u_1 + ... (one elementwise torch add per message: the reference's
`val[i] += upd[i]` per message, numeric_store_row.hpp:177-185, in message order).

C4: one owner shard of the 10M x 1024 table as the exchange delivers it — world = 8
per-source messages of width-1024 records applied in source order — bit-exact against
the oracle at a reduced row count, and a shard whose first message exceeds 4 GiB (the
v2 kernel's 64-bit record addressing) bit-exact against the in-order torch sum.
"""
import numpy as np
import pytest

torch = pytest.importorskip("torch")

import parameter_server_amd as psa
from parameter_server_amd import wire
from oracle.oracle import OracleServer, DENSE, F32

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module", autouse=True)
def _gpu(built_lib, oracle_lib):
    if not torch.cuda.is_available():
        pytest.skip("no GPU")


def _in_order_reference(table0, msgs):
    """msgs: [(slots int64 cuda, upd f32 cuda [n, cap])] in message order."""
    ref = table0.clone()
    for slots, upd in msgs:
        ref[slots] = ref[slots] + upd          # one rounding per element per message
    return ref


def _apply_device(srv, streams, bgs, ver):
    srv.apply_device([(s.data_ptr(), s.numel(), bg, ver) for s, bg in zip(streams, bgs)])
    srv.sync()


def test_c2_full_size_bit_exact():
    rows, cap, B = 1 << 20, 256, 8
    g = torch.Generator(device="cuda").manual_seed(2024)
    table0 = torch.randn(rows, cap, device="cuda", generator=g) * 0.1
    bgs = [100 + b for b in range(B)]
    srv = psa.Server(0, 1, bgs)
    srv.set_stream(torch.cuda.current_stream().cuda_stream)
    srv.CreateTable(1, psa.TableInfo(row_kind=psa.ROW_DENSE, dtype=F32, row_capacity=cap, max_rows=rows))
    srv.load_rows(1, 0, None, on_device_ptr=table0.data_ptr(), num_rows=rows)
    ref = table0
    for ver in range(2):                         # two steps: the index is restored between calls
        streams, msgs = [], []
        for b in range(B):
            perm = torch.randperm(rows, device="cuda", generator=g)
            upd = torch.randn(rows, cap, device="cuda", generator=g) * 0.01
            streams.append(wire.dense_stream_torch(1, perm.to(torch.int32), upd))
            msgs.append((perm, upd))
        torch.cuda.synchronize()
        _apply_device(srv, streams, bgs, ver)
        ref = _in_order_reference(ref, msgs)
        del streams, msgs
    got = torch.empty_like(ref)
    from parameter_server_amd import _abi
    assert _abi.load().psx_table_read_rows(srv.handle, 1, 0, rows, got.data_ptr(), 1) == 0
    torch.cuda.synchronize()
    assert torch.equal(got.view(torch.int32), ref.view(torch.int32))
    srv.close()


def test_c4_shard_world8_bit_exact_vs_oracle():
    """Owner 3 of an 8-way row-range sharding (rows [3*S, 4*S)): eight per-source messages
    of full-coverage width-1024 records in random row order, applied in source order in
    one fused call, bit-exact against the oracle's sequential apply."""
    rng = np.random.RandomState(404)
    S, cap, world, owner = 1500, 1024, 8, 3
    base = owner * S
    bgs = [100 + w for w in range(world)]
    srv = psa.Server(0, 1 + owner, bgs)
    srv.CreateTable(1, psa.TableInfo(row_kind=psa.ROW_DENSE, dtype=F32, row_capacity=cap,
                                     row_offset=base, max_rows=S))
    orc = OracleServer(bgs)
    orc.create_table(1, DENSE, F32, cap)
    init = rng.normal(0, 0.1, size=(S, cap)).astype(np.float32)
    srv.load_rows(1, base, init)
    orc.load_dense_rows(1, base, init)
    streams = [wire.dense_stream_np(1, (rng.permutation(S) + base).astype(np.int32),
                                    rng.normal(0, 0.01, size=(S, cap)).astype(np.float32)) for _ in range(world)]
    dev = [torch.from_numpy(s).cuda() for s in streams]
    torch.cuda.synchronize()
    _apply_device(srv, dev, bgs, 0)
    for s, bg in zip(streams, bgs):
        assert orc.apply_stream(s, bg, 0) == 0
    assert np.array_equal(srv.read_rows(1, base, S).view(np.uint32),
                          orc.read_dense_rows(1, base, S).view(np.uint32))


def test_v3_message_between_2_and_4_gib_bit_exact():
    """dense_apply_v3 addresses records by a 32-bit unsigned offset from an SGPR base (the
    saddr form).  A 2.5 GiB message of width-1024 records puts the offsets of its last
    ~130K records past 2^31, where a sign-extended offset would address 4 GiB below the
    message (the round-5 fault of a removed scalar-load variant came from exactly that
    kind of extension).  One such message plus seven of 100K records, through
    both placements (row ids from the stream: apply_device; producer record-row lists:
    apply_indexed_rows, whose row-id check reads at `base + i*stride - 4`), must be
    bit-exact against the in-order sum, and v3 must be the kernel taken
    (PSX_STAT_DENSE_LAST).  Reference: the int32 stream cursor this product lifts,
    serialized_oplog_reader.hpp:137."""
    from parameter_server_amd import _abi
    L = _abi.load()
    PSX_STAT_DENSE_LAST = 24
    S, cap = 655_360, 1024
    g = torch.Generator(device="cuda").manual_seed(2025)
    table0 = torch.randn(S, cap, device="cuda", generator=g) * 0.1
    bgs = [100 + w for w in range(8)]
    srv = psa.Server(0, 1, bgs)
    srv.set_stream(torch.cuda.current_stream().cuda_stream)
    srv.CreateTable(1, psa.TableInfo(row_kind=psa.ROW_DENSE, dtype=F32, row_capacity=cap, max_rows=S))
    srv.load_rows(1, 0, None, on_device_ptr=table0.data_ptr(), num_rows=S)
    streams, msgs, lists = [], [], []
    for w in range(8):
        # 100K records each: over 2 records per row in all, so the auto selection takes v3
        # (sparse_coverage would pick v4 below that)
        n = S if w == 0 else 100_000
        perm = torch.randperm(S, device="cuda", generator=g)[:n]
        upd = torch.randn(n, cap, device="cuda", generator=g) * 0.01
        streams.append(wire.dense_stream_torch(1, perm.to(torch.int32), upd))
        lists.append(perm.to(torch.int32))
        msgs.append((perm, upd))
    big = streams[0].numel()
    assert (1 << 31) + (256 << 20) < big < (4 << 30) - (64 << 10)
    assert (S - 1) * (4 + 4 * cap) > (1 << 31)       # the last records' offsets have bit 31 set
    torch.cuda.synchronize()
    L.psx_debug_set_variant(PSX_STAT_DENSE_LAST, 0)
    _apply_device(srv, streams, bgs, 0)
    assert L.psx_debug_get_variant(PSX_STAT_DENSE_LAST) == 3, "v3 not taken (walked call)"
    L.psx_debug_set_variant(PSX_STAT_DENSE_LAST, 0)
    srv.apply_indexed_rows([(s.data_ptr(), s.numel(), bg, 1) for s, bg in zip(streams, bgs)],
                           [r.data_ptr() for r in lists])
    srv.sync()
    assert L.psx_debug_get_variant(PSX_STAT_DENSE_LAST) == 3, "v3 not taken (record-row call)"
    del streams, lists
    ref = _in_order_reference(_in_order_reference(table0, msgs), msgs)
    del msgs, table0
    got = torch.empty_like(ref)
    assert L.psx_table_read_rows(srv.handle, 1, 0, S, got.data_ptr(), 1) == 0
    torch.cuda.synchronize()
    ndiff = int((got.view(torch.int32) != ref.view(torch.int32)).sum().item())
    assert ndiff == 0, f"{ndiff} values differ"
    srv.close()


def test_c4_stream_over_4gib_bit_exact():
    """A C4 shard message larger than 4 GiB (1.1M width-1024 records = 4.5 GB) followed by
    seven smaller ones: v3's 32-bit record offsets cannot address it, so the runtime takes
    the v2 kernel; still bit-exact against the in-order sum."""
    S, cap = 1_100_000, 1024
    g = torch.Generator(device="cuda").manual_seed(77)
    table0 = torch.randn(S, cap, device="cuda", generator=g) * 0.1
    bgs = [100 + w for w in range(8)]
    srv = psa.Server(0, 1, bgs)
    srv.set_stream(torch.cuda.current_stream().cuda_stream)
    srv.CreateTable(1, psa.TableInfo(row_kind=psa.ROW_DENSE, dtype=F32, row_capacity=cap, max_rows=S))
    srv.load_rows(1, 0, None, on_device_ptr=table0.data_ptr(), num_rows=S)
    streams, msgs = [], []
    for w in range(8):
        n = S if w == 0 else 50_000
        perm = torch.randperm(S, device="cuda", generator=g)[:n]
        upd = torch.randn(n, cap, device="cuda", generator=g) * 0.01
        streams.append(wire.dense_stream_torch(1, perm.to(torch.int32), upd))
        msgs.append((perm, upd))
    assert streams[0].numel() > (4 << 30)
    torch.cuda.synchronize()
    _apply_device(srv, streams, bgs, 0)
    ref = _in_order_reference(table0, msgs)
    del streams, msgs
    got = torch.empty_like(ref)
    from parameter_server_amd import _abi
    assert _abi.load().psx_table_read_rows(srv.handle, 1, 0, S, got.data_ptr(), 1) == 0
    torch.cuda.synchronize()
    assert torch.equal(got.view(torch.int32), ref.view(torch.int32))
    srv.close()
