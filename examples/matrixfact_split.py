"""C1 (BASELINE.json configs[0]): a small-scale restatement of apps/matrixfact's
matrixfact_split on one client with 2 worker threads, driving a row-update server
through the reference's server interface (Server::ApplyOpLogUpdateVersion and the push
of dirty rows).

What it restates (reference file:line):
  * data: one data_split partition `<name>.0` = size_t nnz, rows, cols; int rows[nnz];
    int cols[nnz]; float vals[nnz] (data_split.cpp:200-217, read by ReadBinaryMatrix,
    matrixfact_split.cpp:62-97), rows sorted;
  * PartitionWorkLoad (matrixfact_split.cpp:99-126): contiguous nnz ranges per worker,
    split on row boundaries;
  * InitMF (:227-253): L rows local, R columns owned by a worker are initialised through
    R_table.DenseBatchInc with N(0, 0.1) values;
  * SgdElement (:180-225): LiRj = L(i,:) R(:,j); grad_coeff = -2 (X_ij - LiRj); per k
    L(i,k) += -step * (grad_coeff R(k,j) + 2 lambda / nnz_per_row L(i,k)), then the R
    update -step * (grad_coeff L(i,k) + 2 lambda / nnz_per_col R(k,j)) goes to
    R_table.DenseBatchInc(j, ...);
  * step_size = init_step_size * step_dec^iter (use_step_dec, :473-476, with the run
    script's single-machine init_step_size 8e-3, step_dec 0.995 and lambda 0.05,
    run_matrixfact_split.sh:50-58); one clock
    per iteration;
  * client side of DenseBatchInc (ssp_consistency_controller.cpp:129-187): the row oplog
    is overwritten on first touch, then accumulated `oplog[c] += u[c]`, and the update is
    applied to the process-cache row at once;
  * on Clock the bg worker packs every row oplog of the table into one ClientSendOpLogMsg
    (ssp_bg_worker.cpp:169-213, dense serialization, rows in ascending id here: the
    reference's libcuckoo order is unspecified) with an incrementing version
    (ssp_bg_worker.cpp:250-257); the server applies it and pushes every dirty row back
    (server.cpp:189-309); the client resets its cached rows to the pushed values
    (UpdateExistingRow with no_oplog_replay, abstract_bg_worker.cpp:775-805).

The schedule is deterministic: worker 0's share, then worker 1's, each iteration (the
reference interleaves two threads; the server sees one message per clock either way,
since ClockConservative sends when the last worker ticks, table_group.cpp:219-234).

`server` is anything with ApplyOpLogUpdateVersion(bytes, size, bg, version) and
push_body() -> bytes (the GPU server, or the CPU checker in the tests)."""
import os
import struct

import numpy as np

from parameter_server_amd import wire


def write_split(path, rows=2000, cols=1000, nnz=10000, seed=1234):
    """One data_split partition file (data_split.cpp:200-217)."""
    rng = np.random.RandomState(seed)
    flat = np.sort(rng.choice(rows * cols, size=nnz, replace=False))
    r = (flat // cols).astype(np.int32)
    c = (flat % cols).astype(np.int32)
    v = rng.uniform(1, 5, size=nnz).astype(np.float32)
    with open(path, "wb") as f:
        f.write(struct.pack("<QQQ", nnz, rows, cols))
        f.write(r.tobytes())
        f.write(c.tobytes())
        f.write(v.tobytes())
    return path


def read_split(path):
    """ReadBinaryMatrix (matrixfact_split.cpp:62-97)."""
    with open(path, "rb") as f:
        nnz, rows, cols = struct.unpack("<QQQ", f.read(24))
        r = np.frombuffer(f.read(4 * nnz), np.int32)
        c = np.frombuffer(f.read(4 * nnz), np.int32)
        v = np.frombuffer(f.read(4 * nnz), np.float32)
    return r, c, v, int(rows), int(cols)


def partition_workload(x_row, workers):
    """PartitionWorkLoad (matrixfact_split.cpp:99-126): partition starts."""
    nnz = x_row.size
    per = nnz // workers
    starts, start = [], 0
    for i in range(workers):
        starts.append(start)
        if i != workers - 1:
            end = start + per
            rid = x_row[end]
            while end < nnz and x_row[end] == rid:
                end += 1
            start = end
    return starts


class Client:
    """One client process: a shared R process cache and the R table's row oplogs."""

    def __init__(self, m, k, table_id=1):
        self.R = {}                   # process cache rows (created by the first push)
        self.oplog = {}               # row oplogs (DenseRowOpLog, capacity K)
        self.K, self.table_id = k, table_id

    def dense_batch_inc(self, j, u):
        if j in self.oplog:
            self.oplog[j] += u        # DenseBatchIncDenseOpLog (:175-187)
        else:
            self.oplog[j] = u.copy()  # OverwriteWithDenseUpdate (:140-141)
        if j in self.R:
            self.R[j] += u            # process-cache apply (:150-159)

    def pack(self):
        """The ClientSendOpLogMsg payload of this clock; resets the oplogs."""
        ids = np.array(sorted(self.oplog), dtype=np.int32)
        if ids.size == 0:
            return np.zeros(0, np.uint8)
        ops = np.stack([self.oplog[j] for j in ids]).astype(np.float32)
        self.oplog = {}
        return wire.dense_stream_np(self.table_id, ids, ops)

    def apply_push(self, body):
        """SerializedRowReader + ResetRowData (serialized_row_reader.hpp:49-93)."""
        for rid, data in wire.parse_push_body(body).get(self.table_id, {}).items():
            self.R[rid] = np.frombuffer(data, np.float32).copy()


def run(server, path, k=16, iters=4, workers=2, bg_id=0, init_step=8e-3, step_dec=0.995, lam=0.05, seed=1234):
    """Returns per-iteration (loss, message, push body) for the given server."""
    x_row, x_col, x_val, n_rows, n_cols = read_split(path)
    starts = partition_workload(x_row, workers)
    ends = starts[1:] + [x_row.size]
    rng = np.random.RandomState(seed)
    L = {i: rng.normal(0, 0.1, size=k).astype(np.float32) for i in np.unique(x_row)}
    cli = Client(n_cols, k)
    per_w = n_cols // workers
    for w in range(workers):       # InitMF: each worker initialises its R columns
        c0, c1 = w * per_w, (n_cols if w == workers - 1 else (w + 1) * per_w)
        for j in range(c0, c1):
            cli.dense_batch_inc(j, rng.normal(0, 0.1, size=k).astype(np.float32))
    version = 0
    msg = cli.pack()
    server.ApplyOpLogUpdateVersion(msg, msg.size, bg_id, version)
    version += 1
    cli.apply_push(server.push_body())
    two_lam = np.float32(lam * 2)
    out = []
    for it in range(iters):
        step = np.float32(init_step * step_dec ** it)       # use_step_dec (:473-476, run script)
        for w in range(workers):
            for a in range(starts[w], ends[w]):
                i, j, xij = int(x_row[a]), int(x_col[a]), x_val[a]
                Li, Rj = L[i], cli.R[j].copy()
                grad_coeff = np.float32(-2) * (xij - np.float32(np.dot(Li, Rj)))
                Li += -(grad_coeff * Rj + two_lam * Li) * step       # nnz_per_row = 1
                upd = -(grad_coeff * Li + two_lam * Rj) * step       # nnz_per_col = 1
                cli.dense_batch_inc(j, upd.astype(np.float32))
        msg = cli.pack()
        server.ApplyOpLogUpdateVersion(msg, msg.size, bg_id, version)
        version += 1
        body = server.push_body()
        cli.apply_push(body)
        pred = np.array([np.dot(L[int(i)], cli.R[int(j)]) for i, j in zip(x_row, x_col)], np.float64)
        out.append((float(np.sum((x_val - pred) ** 2)), msg, bytes(body)))
    return out


if __name__ == "__main__":
    import sys
    import tempfile
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import parameter_server_amd as psa

    class GpuServer:
        def __init__(self, cols, k):
            self.s = psa.Server(0, 1, [0])
            self.s.CreateTable(1, psa.TableInfo(row_kind=psa.ROW_DENSE, dtype=psa.F32, row_capacity=k, max_rows=cols))

        def ApplyOpLogUpdateVersion(self, *a):
            self.s.ApplyOpLogUpdateVersion(*a)

        def push_body(self):
            return bytes(self.s.serialize_dirty(clear=True))

    with tempfile.TemporaryDirectory() as d:
        p = write_split(os.path.join(d, "mf.0"))
        for it, (loss, msg, body) in enumerate(run(GpuServer(1000, 16), p)):
            print(f"iter {it + 1}: L2 loss {loss:.3f}  message {msg.size} B  push {len(body)} B")
