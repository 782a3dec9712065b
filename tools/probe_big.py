"""Diagnosis: one near-2-GiB dense message (a) applied directly, (b) self-exchanged over a
one-rank RCCL communicator, (c) both concurrently on separate streams."""
import faulthandler
import sys
import time

import torch

sys.path.insert(0, ".")
import parameter_server_amd as psa
from parameter_server_amd import wire
from parameter_server_amd.exchange import Exchange

faulthandler.dump_traceback_later(float(sys.argv[2]) if len(sys.argv) > 2 else 60, exit=True)
mode = sys.argv[1]
rows, cap = 600_000, 1024
n = int(sys.argv[3]) if len(sys.argv) > 3 else 523_776
g = torch.Generator(device="cuda").manual_seed(1)
perm = torch.randperm(rows, generator=g, device="cuda")[:n].to(torch.int32)
upd = torch.randn(n, cap, generator=g, device="cuda") * 0.01
msg = wire.dense_stream_torch(1, perm, upd)
print("message bytes", msg.numel(), flush=True)
srv = psa.Server(0, 1, [100])
srv.CreateTable(1, psa.TableInfo(row_kind=psa.ROW_DENSE, dtype=psa.F32, row_capacity=cap, max_rows=rows))
t0 = time.perf_counter()
if mode == "apply":
    srv.apply_device([(msg.data_ptr(), msg.numel(), 100, 0)])
    srv.sync()
    got = torch.from_numpy(srv.read_rows(1, 0, rows)).cuda()
    exp = torch.zeros(rows, cap, device="cuda")
    exp[perm.long()] += upd
    print("apply ok", time.perf_counter() - t0, "equal", bool(torch.equal(got, exp)), flush=True)
elif mode == "xchg":
    xc = Exchange(0)
    recv, rs = xc.alltoall(msg, [msg.numel()])
    torch.cuda.synchronize()
    print("xchg ok", time.perf_counter() - t0, bool(torch.equal(recv, msg)), flush=True)
elif mode == "both":
    xc = Exchange(0)
    s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
    srv.set_stream(s1.cuda_stream)
    recv = torch.empty_like(msg)
    srv.apply_device([(msg.data_ptr(), msg.numel(), 100, 0)])
    xc.streams_into(msg, [msg.numel()], recv, [msg.numel()], s2.cuda_stream)
    srv.sync()
    print("apply done", time.perf_counter() - t0, flush=True)
    s2.synchronize()
    print("both ok", time.perf_counter() - t0, bool(torch.equal(recv, msg)), flush=True)
