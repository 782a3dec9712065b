"""The Server methods parameter_server_amd.ServerThread calls, over the CPU oracle — the
checker side of the ServerThread replays (test infrastructure only)."""
from oracle.oracle import OracleServer, DENSE


class OracleBackend:
    """The Server methods ServerThread calls, over the oracle."""

    def __init__(self, bgs, num_clients):
        self.o = OracleServer(bgs)
        self.num_clients = num_clients
        self.tables = []

    def create(self, tid, kind, dt, cap, dense_serialized=True, version_maintain=False, adarevision=None):
        """adarevision: dict(init_step_size, gaussian_init, old_grad_upper_bound) attaches
        AdaRevisionServerTableLogic (push_clients = this backend's clients)."""
        self.o.create_table(tid, kind, dt, cap if kind == DENSE else 0, oplog_dense_serialized=dense_serialized,
                            version_maintain=version_maintain)
        if adarevision is not None:
            assert self.o.set_adarevision(tid, push_clients=self.num_clients, **adarevision) == 0
        self.tables.append(tid)

    def ApplyOpLogUpdateVersion(self, payload, size, bg, version):
        assert self.o.apply_stream(payload, bg, version) == 0

    def ClockUntil(self, bg, clock):
        return self.o.clock_until(bg, clock)

    def GetMinClock(self):
        return self.o.min_clock()

    def subscribe(self, tid, rows, client):
        for r in rows:
            self.o.subscribe(tid, int(r), client)

    def serialize_rows(self, tid, rows):
        return self.o.serialize_records(tid, rows)

    def row_sent(self, tid, rows, n):
        for r in rows:
            assert self.o.row_sent(tid, int(r), n) == 0

    def serialize_push(self, clear=True):
        return self.o.serialize_push(self.tables, self.num_clients, clear=clear)
