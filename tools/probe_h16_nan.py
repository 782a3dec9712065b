"""Probe: does the gfx950 f16->f32 conversion keep NaN payloads, and do rows after
`row += u` match the payload-exact decompression bit for bit (variants 1 vs 2)?"""
import numpy as np
import torch
import parameter_server_amd as psa
from parameter_server_amd import wire, _abi

h = np.array([0x7e01, 0xfd55, 0x7c01, 0x7dff, 0xfe00, 0x7fff, 0x3c00, 0x0001], np.uint16)
t = torch.from_numpy(h.view(np.int16)).cuda().view(torch.float16).float().view(torch.int32).cpu().numpy()
print("hw cvt:", [hex(int(x)) for x in t.view(np.uint32)])
L = _abi.load()
rows, cap = 4, 8
res = {}
for v in (0, 2):
    L.psx_debug_set_variant(4, v)
    srv = psa.Server(0, 1, [100] + list(range(101, 108)))
    srv.CreateTable(1, psa.TableInfo(row_kind=0, dtype=0, row_capacity=cap, max_rows=rows, row_oplog_type=3))
    srv.load_rows(1, 0, np.array([[1.5] * cap, [np.nan] * cap, [0.0] * cap, [-2.0] * cap], np.float32))
    msgs = [torch.from_numpy(wire.dense_variant_stream_np(1, np.arange(rows, dtype=np.int32), np.tile(h, (rows, 1)), f16=True)).cuda()
            for _ in range(8)]
    torch.cuda.synchronize()
    srv.apply_device([(m.data_ptr(), m.numel(), 100 + b, 0) for b, m in enumerate(msgs)])
    srv.sync()
    res[v] = srv.read_rows(1, 0, rows).view(np.uint32)
    srv.close()
L.psx_debug_set_variant(4, 0)
print("rows v0:", [[hex(x) for x in r] for r in res[0]])
print("identical after add:", bool(np.array_equal(res[0], res[2])))
