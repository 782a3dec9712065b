"""Headline benchmark: row-update apply GB/s (device-resident), dense f32 rows.

Workload (BASELINE.json configs[1]): one DenseRow<float> table of
2^20 rows x 256 cols per GPU (initialised N(0, 0.1)); one step = applying B = 8 worker
batches, each a full Appendix-A stream (ClientSendOpLogMsg payload) holding one dense
record per row in a per-batch random row order, updates N(0, 0.01).  Streams and table
are resident in HBM before the timed region.  Synthetic data, generated on the GPU.

Records are placed from the producer's record-row lists (psx_apply_indexed_rows: the rows
psx_pack_stream_indexed packed, 4 B per record; every record's row id is still checked
against its row inside the apply) with each call's index stage overlapping the previous
call's apply; the same messages through the walked path (row ids read from the stream,
psx_apply_streams_device) are timed after it and reported as `walked` (--walked: only that).

Algorithmic bytes per step: sum_b (20 + N_b*(4 + 4R)) + 2 * N_touched * 4R,
plus 4 * N_b per listed message (N_b = N at full density; --density 0.125 gives the §8(d)
partial-coverage variant).
value = bytes of all ranks / max-over-ranks wall time.  Multi-GPU: each rank owns a
2^20-row shard (row range) and receives its own already-split batches, as the reference
client splits oplogs by owning server (abstract_bg_worker.cpp:590-649): no collective,
weak scaling.

After the timed region the bare run (no variant flags) also records the PCIe-inclusive
rate and C3 walked / pipelined / indexed (N = 1, child processes), or the exchange-bearing
step (N > 1: each rank's batch spans every shard, one RCCL all-to-all over xGMI, then the
owners' fused applies) — `--no-extras` leaves them out.

cpu_baseline: the CPU oracle (restated Server::ApplyOpLogUpdateVersion loop, one
thread = one reference server thread) on a bounded sample of the same workload.
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

EXCHANGE_TIMEOUT_S = 600   # N > 1: the exchange extras are abandoned (headline kept, exit 3) past this
HBM_PEAK_GBS = 8000.0   # MI355X HBM3E spec (MI355X_MICROARCH.md, chip-level parameters)
PMC_JSON = os.path.join(ROOT, "profiles", "r06", "pmc_dense_apply.json")


def kernel_signature():
    """Identity of the measured dense-apply code: a hash of the sources that define the
    kernels and their launch policy and of the compile flags.  A PMC JSON carries the
    signature it was measured on; traffic from another signature is not reported."""
    import hashlib
    import re
    h = hashlib.sha256()
    csrc = os.path.join(ROOT, "parameter_server_amd", "csrc")
    h.update(open(os.path.join(csrc, "psx_kernels.hip"), "rb").read())
    # of psx_device.hpp only what the dense kernels take: the shared device constants and
    # structs up to DenseArgs (the ordered path's and the walk's structs may change freely)
    dev = open(os.path.join(csrc, "psx_device.hpp")).read()
    m = re.search(r"^struct DenseArgs \{.*?^\};", dev, re.S | re.M)
    h.update(dev[:m.end()].encode() if m else dev.encode())
    for line in open(os.path.join(csrc, "Makefile")):
        if line.startswith("HIPFLAGS") or line.startswith("           -"):
            h.update(line.encode())
    return h.hexdigest()[:16]


C3_PMC_JSON = os.path.join(ROOT, "profiles", "r06", "pmc_c3.json")


def c3_kernel_signature():
    """Identity of the code a C3 step runs (walk, ordered path, decode, the device structs,
    the flags): the C3 PMC JSON is reported only on the tree it was measured on."""
    import hashlib
    h = hashlib.sha256()
    csrc = os.path.join(ROOT, "parameter_server_amd", "csrc")
    for f in ("psx_walk.hip", "psx_ordered.hip", "psx_kernels.hip", "psx_device.hpp", "psx_scan.hpp"):
        h.update(open(os.path.join(csrc, f), "rb").read())
    for line in open(os.path.join(csrc, "Makefile")):
        if line.startswith("HIPFLAGS") or line.startswith("           -"):
            h.update(line.encode())
    return h.hexdigest()[:16]


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=20)
    p.add_argument("--warmup", type=int, default=3)
    p.add_argument("--rows", type=int, default=1 << 20, help="rows per GPU shard")
    p.add_argument("--cols", type=int, default=256)
    p.add_argument("--variant", action="append", default=[], metavar="ID=VALUE",
                   help="A/B runs: psx_debug_set_variant(ID, VALUE) before anything runs (include/psx_debug.h)")
    p.add_argument("--batches", type=int, default=8)
    p.add_argument("--cpu-seconds", type=float, default=12.0,
                   help="target CPU time of the cpu_baseline sample (0 disables)")
    p.add_argument("--cpu-rows", type=int, default=1 << 18,
                   help="rows of a generated cpu_baseline sample (configurations that do not hand the baseline "
                        "their own messages; the C2 line times the oracle on the full C2 messages)")
    p.add_argument("--cpu-threads", type=int, default=0,
                   help="cap on the cpu_baseline's server threads (0: every usable core -- the affinity mask, "
                        "cgroup quota and OMP_NUM_THREADS; the GPU box's share is 16)")
    p.add_argument("--pmc-json", default=PMC_JSON,
                   help="per-launch HBM bytes of dense_apply from the rocprofv3 --pmc passes "
                        "(tools/pmc_summary.py); used for roofline.traffic on the default C2 configuration")
    p.add_argument("--f16-records", action="store_true",
                   help="C2 with kDenseRowOpLogFloat16 records (binary16 payloads, row_oplog_type 3)")
    p.add_argument("--workload", default="c2", choices=["c2", "c3", "c4", "c4shard", "c5"],
                   help="c2: dense f32 headline (default); c3: LDA-style sparse int sorted-map rows; "
                        "c4: 10M x 1K dense table sharded over ranks with an all-to-all exchange; "
                        "c4shard: one GPU's 1.25M-row shard of C4 with its 8 worker messages; "
                        "c5: mixed dense + sparse clocks under SSPPush")
    p.add_argument("--c4-rows", type=int, default=10_000_000, help="C4 total rows (all shards)")
    p.add_argument("--c5-gloo", action="store_true",
                   help="C5 with WORLD_SIZE > 1 over gloo (no collective is on C5's data path; the tests put 2 "
                        "ranks on one GPU)")
    p.add_argument("--c5-dump", default=None,
                   help="C5: every rank writes its shard and applied message order to this directory")
    p.add_argument("--adarevision", action="store_true",
                   help="C2 through the AdaRevision server-table logic (adarevision_server_table_logic.cpp): "
                        "per element the adaptive step on accum/z/z_max state beside every row")
    p.add_argument("--density", type=float, default=1.0,
                   help="C2 fraction of rows each batch covers (SURVEY §8(d) C2 variant: 0.125)")
    p.add_argument("--indexed", action="store_true",
                   help="C3 through psx_apply_indexed: producer record indexes replace the sequential sparse walk")
    p.add_argument("--walked", action="store_true",
                   help="C2 through psx_apply_streams_device only: every record's row id read from the stream to "
                        "place it (the default run measures the producer record-row path, psx_apply_indexed_rows, "
                        "and reports this walked path beside it)")
    p.add_argument("--skip-walked", action="store_true",
                   help="do not time the walked path after the record-row run (profiler passes: every "
                        "dense_apply launch then belongs to the measured configuration)")
    p.add_argument("--importance", action="store_true",
                   help="C2 with importance accumulation (SSPAggr RelativeMagnitude tables)")
    p.add_argument("--pcie", action="store_true",
                   help="also time the host-buffer form: pinned H2D of the 8 messages + apply + D2H of "
                        "every (dirty) row, i.e. the rate including PCIe (reported, never `value`)")
    p.add_argument("--no-extras", dest="extras", action="store_false",
                   help="plain C2 line only: no PCIe-inclusive pass, no C3 (N = 1), no exchange step (N > 1) "
                        "after the timed region (profiler passes)")
    p.add_argument("--master-port", type=int, default=29531,
                   help="rendezvous port when bench.py launches its own ranks (--gpus N, WORLD_SIZE unset)")
    p.add_argument("--selftest-exchange", action="store_true",
                   help="run exchange_measure's orchestration and parity check over gloo on the CPU "
                        "(CpuShardExchange in place of the device path): the CPU test of the N > 1 extras")
    p.add_argument("--selftest-reverse", action="store_true", help=argparse.SUPPRESS)   # the check's negative test
    p.add_argument("--selftest-device", action="store_true",
                   help="with --selftest-exchange: every rank on cuda:0 with the real device path "
                        "(ShardExchange: psx split, apply) and the bytes crossing over gloo (GlooExchange) "
                        "-- the multi-rank GPU test on a one-GPU box")
    p.add_argument("--selftest-launch", action="store_true",
                   help="exercise only the multi-rank harness (rank launch, barriers, max-over-ranks timing, "
                        "the JSON line) over gloo with a no-op step: the CPU test of --gpus N")
    return p.parse_args()


def run_child(flags, timeout=300):
    """One bench.py run as a child process (this process keeps its GPU context; the child
    starts its own): returns the child's JSON line."""
    import subprocess
    out = subprocess.run([sys.executable, os.path.abspath(__file__)] + flags, capture_output=True, text=True,
                         timeout=timeout, env={k: v for k, v in os.environ.items()
                                               if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")})
    lines = [l for l in out.stdout.splitlines() if l.startswith("{")]
    if out.returncode != 0 or not lines:
        raise RuntimeError(f"child rc={out.returncode}: {out.stderr[-300:]}")
    return json.loads(lines[-1])


def launch_ranks(args):
    """`python bench.py --gpus N` without a launcher: start N ranks, one per GPU, through
    torch.distributed.run as a CHILD process (this process has touched no GPU) and exit
    with its status.  Rank 0 prints the JSON line."""
    import subprocess
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
           "--master-addr", "127.0.0.1", f"--master-port={args.master_port}", os.path.abspath(__file__)]
    cmd += sys.argv[1:]
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    return subprocess.run(cmd, env=env).returncode


def selftest_launch(args):
    """The harness of the N-rank bench with a no-op step (gloo, CPU): barrier + max-over-
    ranks timing around K steps, rank 0 prints one JSON line with n_gpus = world."""
    import torch
    import torch.distributed as dist
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    if world > 1:
        dist.init_process_group("gloo")
    for _ in range(args.warmup):
        pass
    if world > 1:
        dist.barrier()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        time.sleep(0.001 * (1 + rank))
    if world > 1:
        dist.barrier()
    el = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([el], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        el = float(t.item())
    if rank == 0:
        print(json.dumps({"metric": "selftest-launch", "value": round(args.steps / el, 3), "unit": "steps/s",
                          "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
                          "ms_per_step": round(el / args.steps * 1e3, 4)}), flush=True)
    if world > 1:
        dist.destroy_process_group()


def cpu_model():
    try:
        with open("/proc/cpuinfo") as f:
            return next((l.split(":", 1)[1].strip() for l in f if l.startswith("model name")), None)
    except OSError:
        return None


def usable_cores():
    """CPUs this process may use and where the figure comes from: its affinity mask, capped
    by a cgroup CPU quota and by OMP_NUM_THREADS (the GPU box runs a job on a 16-CPU share
    of its host and says so there; nproc / os.cpu_count() show the whole machine)."""
    info = {"nproc": os.cpu_count()}
    n = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    info["affinity"] = n
    quota = None
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if q != "max":
            quota = max(1, int(q) // int(per))
    except (OSError, ValueError):
        try:
            q = int(open("/sys/fs/cgroup/cpu/cpu.cfs_quota_us").read())
            per = int(open("/sys/fs/cgroup/cpu/cpu.cfs_period_us").read())
            if q > 0:
                quota = max(1, q // per)
        except (OSError, ValueError):
            pass
    info["cgroup_quota"] = quota
    omp = os.environ.get("OMP_NUM_THREADS")
    info["omp_num_threads"] = int(omp) if omp and omp.isdigit() else None
    T = min(x for x in (n, quota, info["omp_num_threads"]) if x)
    return max(1, T), info


def cpu_baseline(args, rows=None, cap=None, host_msgs=None, base=0):
    """Oracle (CPU restatement of the reference apply loop) run as T server threads: rows
    are sharded row_id % T (the reference's comm-channel placement, context.hpp:291-304) and
    each thread applies its own shard's messages, as T reference ServerThreads would (the
    client already splits its oplog per server, abstract_bg_worker.cpp:590-649).  ctypes
    releases the GIL, so shards run in parallel.  A single-thread pass (one reference server
    thread) is timed beside it.  With host_msgs (the C2 run's own messages, in host memory)
    the sample is the whole C2 configuration; otherwise a generated sample of `rows` rows."""
    import numpy as np
    from concurrent.futures import ThreadPoolExecutor
    from oracle.oracle import OracleServer, DENSE, F32
    from parameter_server_amd import wire
    B = args.batches
    if host_msgs is not None:
        rows, cap = args.rows, args.cols
    else:
        rows, cap = rows or args.cpu_rows, cap or args.cols
    T, tinfo = usable_cores()
    if args.cpu_threads:
        T = min(T, args.cpu_threads)
    rng = np.random.default_rng(1234)
    init = rng.standard_normal((rows, cap), dtype=np.float32) * np.float32(0.1)
    recs = []          # per batch: the records as int32 [n, 1 + cap] (row id, then the payload bits)
    if host_msgs is not None:
        for m in host_msgs:
            recs.append(m[20:].view(np.int32).reshape(-1, 1 + cap))
    else:
        for b in range(B):
            r = np.random.default_rng(1235 + b)
            perm = r.permutation(rows).astype(np.int32)
            upd = r.standard_normal((rows, cap), dtype=np.float32) * np.float32(0.01)
            recs.append(wire.dense_stream_np(1, perm, upd)[20:].view(np.int32).reshape(-1, 1 + cap))
            del upd
    bgs = list(range(100, 100 + B))

    def shard_msg(b, sel):
        r = recs[b] if sel is None else recs[b][sel]
        hdr = np.array([1, 1, 4, 0, r.shape[0]], np.int32)   # one table, update_size 4, num_rows
        return np.concatenate([hdr.view(np.uint8), r.view(np.uint8).reshape(-1)])

    def timed_run(nthreads, seconds):
        shards = []
        for t in range(nthreads):
            o = OracleServer(bgs)
            o.create_table(1, DENSE, F32, cap)
            if args.adarevision:
                assert o.set_adarevision(1, init_step_size=0.1, gaussian_init=False) == 0
            o.load_dense_rows(1, base + t, init[t::nthreads], stride=nthreads)
            msgs = []
            for b in range(B):
                if nthreads == 1 and host_msgs is not None:
                    msgs.append(host_msgs[b])
                else:
                    msgs.append(shard_msg(b, None if nthreads == 1 else ((recs[b][:, 0] - base) % nthreads) == t))
            shards.append((o, msgs))
        step_bytes = sum(m.size for _, ms in shards for m in ms) + (8 if args.adarevision else 2) * rows * cap * 4

        def one(t, ver):
            o, msgs = shards[t]
            for b in range(B):
                assert o.apply_stream_once(msgs[b], bgs[b], ver) == 0

        steps, elapsed = 0, 0.0
        with ThreadPoolExecutor(nthreads) as ex:
            list(ex.map(one, range(nthreads), [0] * nthreads))      # untimed warm-up step
            while elapsed < seconds or steps == 0:
                t0 = time.perf_counter()
                list(ex.map(one, range(nthreads), [steps + 1] * nthreads))
                elapsed += time.perf_counter() - t0
                steps += 1
        for o, _ in shards:
            o.close()
        return step_bytes * steps / elapsed / 1e9, steps, elapsed

    v1, n1, e1 = timed_run(1, args.cpu_seconds / 3)
    vt, nt, et = timed_run(T, args.cpu_seconds * 2 / 3) if T > 1 else (v1, n1, e1)
    what = (f"the C2 run's own {B} messages, copied to the host" if host_msgs is not None else
            "a generated sample")
    return {"value": round(vt, 3), "unit": "GB/s", "cores": T, "kind": "port", "cpu_model": cpu_model(),
            "single_thread_GBps": round(v1, 3), "cores_source": tinfo,
            "sample": f"{rows} rows x {cap} f32, {B} batches/step ({what}); {T} threads = the usable cores "
                      f"(affinity {tinfo['affinity']}, cgroup quota {tinfo['cgroup_quota']}, OMP_NUM_THREADS "
                      f"{tinfo['omp_num_threads']}; nproc {tinfo['nproc']} counts the whole host), rows % {T} "
                      f"shards: {nt} steps in {et:.1f} s; 1 thread (one reference server thread): {n1} steps in "
                      f"{e1:.1f} s (oracle/psx_oracle.c restatement of server.cpp:120-179, single pass: each record "
                      f"checked as it is reached and applied, the reference's loop shape, orc_apply_stream_once)"}


_C3_CACHE = {}


def c3_streams(rows=100_000, K=1024, B=8, per_batch=10_000, seed=1234, with_records=False):
    """SortedVectorMapRow<int32> rows, K columns; B batches of per_batch
    distinct Zipf(s=1) rows, nnz uniform [1, 32], ascending unique columns, values
    +-{1..3} (first batch positive)."""
    import numpy as np
    from parameter_server_amd import wire
    key = (rows, K, B, per_batch, seed)
    if key in _C3_CACHE:        # the default run measures walked and indexed on the same batches
        streams, nupd, batches = _C3_CACHE[key]
        return (streams, nupd, batches) if with_records else (streams, nupd)
    rng = np.random.RandomState(seed)
    p = 1.0 / np.arange(1, rows + 1)
    p /= p.sum()
    streams, nupd, batches = [], 0, []
    for b in range(B):
        ids = rng.choice(rows, size=per_batch, replace=False, p=p)
        ks = rng.randint(1, 33, size=per_batch)
        recs = []
        for rid, k in zip(ids, ks):
            cols = np.sort(rng.choice(K, size=k, replace=False)).astype(np.int32)
            sign = 1 if b == 0 else rng.choice([-1, 1], size=k)
            recs.append((int(rid), cols, (rng.randint(1, 4, size=k) * sign).astype(np.int32)))
        nupd += int(ks.sum())
        streams.append(wire.sparse_stream_np(3, 4, recs))
        batches.append(recs)
    _C3_CACHE[key] = (streams, nupd, batches)
    if with_records:
        return streams, nupd, batches
    return streams, nupd


C3_LATENCY_JSON = os.path.join(ROOT, "profiles", "r02", "c3_inc_latency.json")
C3_WAVES_PER_SIMD = {4: 7, 16: 3}   # ordered_apply_reg_kernel<int32, sorted, J> occupancy (-Rpass-analysis)


def c3_model(batches, rows, K, apply_ms, warmup=3, steps=20, split=3):
    """The sorted-map apply's bound ("C3 bound").  A row's records are one
    dependent chain in one wave: each record's found keys (a chunk of <= 64 columns) are
    added at once (found_run), each new key is one LinearSearchAndMove insert.  So a row
    costs t_r = R_r x Lrec(n_r) + I_r x Lins(n_r): R_r records and I_r inserts per step at
    image size n_r, Lrec / Lins the measured latencies of a lone wave on the kernel the row
    takes (tools/probe_inc_latency.py -> profiles/r02/c3_inc_latency.json).  I_r is exact
    for the timed steps: the bench repeats the same batches, so the value of (row, col)
    before its k-th Inc of step s is s x S + P_k (S its net per step, P_k the partial sum
    before the Inc in message order), and the Inc inserts iff that is 0.  Rows are
    independent waves, w of them resident per SIMD (7 for the 256-entry image, 3 for the
    1,024-entry one), 1,024 SIMDs:
        T >= max( max_r t_r ,  sum_r t_r / (w_r x 1024) )
    (critical path vs latency-interleave throughput; optimistic: no issue contention)."""
    import numpy as np
    if not os.path.exists(C3_LATENCY_JSON):
        return None
    js = json.load(open(C3_LATENCY_JSON))
    if "found_rec_ns" not in js:
        return None

    def curve(name):
        lat = js[name]
        xs = np.array(sorted(int(k) for k in lat), dtype=np.float64)
        return xs, np.array([max(lat[str(int(x))], 0.0) for x in xs], dtype=np.float64)
    r = np.array([rid for recs in batches for rid, _, _ in recs], np.int64)
    rc = np.concatenate([np.full(len(c), rid, np.int64) for recs in batches for rid, c, _ in recs])
    c = np.concatenate([c for recs in batches for _, c, _ in recs]).astype(np.int64)
    v = np.concatenate([v for recs in batches for _, _, v in recs]).astype(np.int64)
    R_r = np.bincount(r, minlength=rows).astype(np.float64)
    k_r = np.bincount(rc, minlength=rows).astype(np.float64)
    key = rc * K + c
    order = np.argsort(key, kind="stable")                     # message order within a key
    ks, vs = key[order], v[order]
    uniq, start, cnt = np.unique(ks, return_index=True, return_counts=True)
    grp = np.repeat(np.arange(uniq.size), cnt)
    csum = np.cumsum(vs)
    base = np.repeat(csum[start] - vs[start], cnt)
    before = csum - vs - base                                  # P_k
    S = np.repeat(np.add.reduceat(vs, start), cnt)
    nz = vs != 0
    ins = np.zeros(vs.size, np.float64)
    zero_S = (S == 0) & nz
    ins[zero_S] = (before[zero_S] == 0)
    m = (S != 0) & nz & (before % np.where(S == 0, 1, S) == 0)
    sk = -before[m] // S[m]
    ins[m] = ((sk >= warmup) & (sk < warmup + steps)) / steps
    I_r = np.bincount(uniq[grp] // K, weights=ins, minlength=rows)
    net = np.add.reduceat(vs, start)
    n_r = np.bincount(uniq[net != 0] // K, minlength=rows).astype(np.float64)
    # the 1,024-entry launch: split form 1 classifies by entries + Incs; the spill forms (2, 3,
    # the default) start a row there only when its image is already > 224 entries (a row that
    # outgrows 256 mid-call spills to it; the timed steps' images stay below 256)
    big = (n_r + k_r > 256) & ((n_r > 224) if split >= 2 else True)
    x16, y16 = curve("found_rec_ns")                           # 1,024-entry image
    x4, y4 = curve("found_small_rec_ns")                       # 256-entry image
    xi, yi = curve("insert_ns")
    t_r = (R_r * np.where(big, np.interp(n_r, x16, y16), np.interp(n_r, x4, y4))
           + I_r * np.interp(n_r, xi, yi)) * 1e-6              # ms
    chain = float(t_r.max())
    tput = float((t_r[~big].sum() / C3_WAVES_PER_SIMD[4] + t_r[big].sum() / C3_WAVES_PER_SIMD[16]) / 1024)
    bound = max(chain, tput)
    hot = int(np.argmax(t_r))
    # measured row throughput: every row's share of the chip at full occupancy (its setup,
    # one record) — the 256-entry launch cannot finish faster than its rows' shares
    share = js.get("row_share_ns")
    rows_bound = float((~big & (R_r > 0)).sum() * share * 1e-6) if share else None
    if rows_bound is not None:
        bound = max(bound, rows_bound)
    return {"bound_ms": round(bound, 4), "critical_path_ms": round(chain, 4), "interleave_ms": round(tput, 4),
            "row_throughput_ms": round(rows_bound, 4) if rows_bound is not None else None,
            "ordered_apply_ms": round(apply_ms, 4), "frac_of_bound": round(bound / apply_ms, 3) if apply_ms else None,
            "rows_touched": int((R_r > 0).sum()), "rows_1024_image": int(big.sum()),
            "inserts_per_step": round(float(I_r.sum()), 1),
            "hot_row": {"records": int(R_r[hot]), "incs": int(k_r[hot]), "inserts": round(float(I_r[hot]), 1),
                        "image": int(n_r[hot])},
            "max_incs_per_row": int(k_r.max()), "max_image": int(n_r.max()),
            "latency_source": os.path.relpath(C3_LATENCY_JSON, ROOT)}


def c3_cpu_baseline(args, batches, nupd, bgs, seconds):
    """The oracle on the same C3 batches as T server threads: rows sharded row % T (the
    reference's comm-channel placement, context.hpp:291-304), each thread applying its
    shard's sub-messages in batch order (the client splits per server,
    abstract_bg_worker.cpp:590-649); ctypes releases the GIL.  One thread beside it."""
    from concurrent.futures import ThreadPoolExecutor
    from oracle.oracle import OracleServer, SORTED_MAP, I32
    from parameter_server_amd import wire
    T = usable_cores()[0]
    if args.cpu_threads:
        T = min(T, args.cpu_threads)

    def timed_run(nthreads, seconds):
        shards = []
        for t in range(nthreads):
            o = OracleServer(bgs)
            o.create_table(3, SORTED_MAP, I32, 0, oplog_dense_serialized=False)
            msgs = [wire.sparse_stream_np(3, 4, [r for r in recs if r[0] % nthreads == t]) for recs in batches]
            shards.append((o, msgs))

        def one(t, v):
            o, msgs = shards[t]
            for b, m in enumerate(msgs):
                assert o.apply_stream_once(m, bgs[b], v) == 0

        n, el, w = 0, 0.0, max(1, args.warmup)
        with ThreadPoolExecutor(nthreads) as ex:
            for v in range(w):        # untimed warm-up steps, as on the GPU
                list(ex.map(one, range(nthreads), [v] * nthreads))
            while el < seconds or n == 0:
                t0 = time.perf_counter()
                list(ex.map(one, range(nthreads), [w + n] * nthreads))
                el += time.perf_counter() - t0
                n += 1
        for o, _ in shards:
            o.close()
        return nupd * n / el / 1e6, n, el

    v1, n1, e1 = timed_run(1, seconds / 3)
    vt, nt, et = timed_run(T, seconds * 2 / 3) if T > 1 else (v1, n1, e1)
    return {"value": round(vt, 3), "unit": "M updates/s", "cores": T, "kind": "port",
            "single_thread": round(v1, 3),
            "sample": f"the same {len(batches)} batches; {T} threads (rows % {T} shards): {nt} steps in {et:.1f} s; "
                      f"1 thread: {n1} steps in {e1:.1f} s (oracle restatement of sorted_vector_map_store.hpp Inc; single "
                      f"pass per message, the reference's loop shape, orc_apply_stream_once)"}


def c3_measure(args, indexed, steps, warmup, cpu_seconds, pipeline=False):
    """Sparse int count rows (C3) on 1 GPU: updates/s (and stream GB/s), the ordered apply
    against its latency model, and (cpu_seconds > 0) the CPU port on the same batches.
    pipeline: psx_ctx_set_pipeline(PSX_PIPELINE_ALL) — each call's decode runs on the side
    stream beside the previous call's apply (the messages are resident before the call)."""
    import numpy as np
    import torch
    import parameter_server_amd as psa
    rows, K, B = 100_000, 1024, args.batches
    streams, nupd, batches = c3_streams(rows, K, B, with_records=True)
    # the product's decode (include/psx_debug.h PSX_VARIANT_DECODE: `--variant 7=0|1`, or
    # PSX_DECODE_WALK in the debug build's environment); the JSON line names the path that ran
    from parameter_server_amd import _abi as _ab
    L = _ab.load()
    decode_variant = L.psx_debug_get_variant(7)
    L.psx_debug_set_variant(8, 0)
    dev = [torch.from_numpy(s).cuda() for s in streams]
    bgs = [100 + b for b in range(B)]
    srv = psa.Server(0, 1, bgs)
    srv.set_stream(torch.cuda.current_stream().cuda_stream)
    srv.CreateTable(3, psa.TableInfo(row_kind=psa.ROW_SORTED_MAP, dtype=psa.I32, row_capacity=K,
                                     oplog_dense_serialized=False, max_rows=rows, max_entries=K))
    if pipeline:
        srv.set_pipeline(2)
    ver = [0]
    idx = None
    if indexed:   # the producer's record index (psx_pack_stream emits the same), built before timing
        from parameter_server_amd import wire as _w
        idx = [torch.from_numpy(_w.stream_record_offsets(s, {3: None}).view(np.int64)).cuda() for s in streams]

    def step():
        msgs = [(d.data_ptr(), d.numel(), bgs[b], ver[0]) for b, d in enumerate(dev)]
        if idx is not None:
            srv.apply_indexed(msgs, [o.data_ptr() for o in idx])
        else:
            srv.apply_device(msgs)
        ver[0] += 1

    for _ in range(warmup):
        step()
    srv.sync()
    # timed region: no events in the stream (an event pair costs a C3 call ~13 us: it drains
    # the queue between launches, profiles/r04/s18 sweep)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        step()
    host_s = time.perf_counter() - t0      # the host's enqueue time for the K calls
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    srv.sync()
    # the apply kernel's launch duration: the same K steps again with events around the
    # apply launches only (timing mode 2)
    srv.timing(2)
    srv.timing_reset()
    for _ in range(steps):
        step()
    srv.sync()
    apply_ms, apply_n = srv.timing_read("ordered_apply")
    # per-kernel breakdown: a separate pass with events around every kernel
    srv.timing(1)
    srv.timing_reset()
    for _ in range(max(3, min(steps, 10))):
        step()
    srv.sync()
    kern = {k: srv.timing_read(k) for k in ("decode_streams", "ordered_prep", "ordered_apply", "finish_call")}
    srv.timing(False)
    srv.close()
    walk_calls = L.psx_debug_get_variant(8)
    if indexed:
        decode = "producer record offsets checked in parallel (decode_streams with offsets)"
    elif walk_calls > 0:
        decode = "window-parallel walk (psx_walk.hip)"
    else:
        decode = "one workgroup per message (decode_streams)"
    stream_bytes = sum(s.size for s in streams)
    model = c3_model(batches, rows, K, apply_ms / max(apply_n, 1), split=L.psx_debug_get_variant(6))
    # algorithmic bytes = the records and headers + a 4-B read and write per
    # distinct (row, col) the step touches
    import numpy as np
    keys = np.unique(np.concatenate([np.int64(rid) * K + c.astype(np.int64) for recs in batches
                                     for rid, c, _ in recs]))
    alg = stream_bytes + 8 * int(keys.size)
    step_s = el / steps
    apply_s = apply_ms / max(apply_n, 1) / 1e3
    roof = {"bound": "hbm", "algorithmic_bytes_per_step": alg, "distinct_row_cols_per_step": int(keys.size),
            "achieved_step_GBps": round(alg / step_s / 1e9, 2), "frac_step": round(alg / step_s / 1e9 / HBM_PEAK_GBS, 4),
            "kernel": "ordered_apply", "achieved": round(alg / apply_s / 1e9, 2) if apply_s else None,
            "kernel_timing": "HIP events around the apply launches over a second pass of the same steps "
                             "(the value's pass runs without events)",
            "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": round(alg / apply_s / 1e9 / HBM_PEAK_GBS, 4) if apply_s else None,
            "traffic": None, "sector_efficiency": None}
    if os.path.exists(C3_PMC_JSON):
        pm = json.load(open(C3_PMC_JSON))
        if pm.get("kernel_signature") == c3_kernel_signature():
            roof["traffic"] = round(pm["bytes_per_step"])
            roof["sector_efficiency"] = round(alg / pm["bytes_per_step"], 4)
            roof["traffic_source"] = os.path.relpath(C3_PMC_JSON, ROOT) + " (L2->fabric request bytes per step, all kernels)"
        else:
            roof["traffic_note"] = f"{os.path.relpath(C3_PMC_JSON, ROOT)} is for another kernel signature"
    cpu = c3_cpu_baseline(args, batches, nupd, bgs, cpu_seconds) if cpu_seconds > 0 else None
    return {
        "metric": "sparse int row-update apply (SortedVectorMapRow<int32>), C3",
        "value": round(nupd * steps / el / 1e6, 3), "unit": "M updates/s",
        "stream_GBps": round(stream_bytes * steps / el / 1e9, 3),
        "n_gpus": 1, "steps": steps, "warmup": warmup,
        "ms_per_step": round(el / steps * 1e3, 4), "higher_is_better": True,
        "host_enqueue_ms_per_step": round(host_s / steps * 1e3, 4),
        "dtype": "int32", "data": "synthetic (Zipf rows, uniform nnz 1..32, values +-1..3)",
        "config": {"workload": f"C3: {rows} rows x K={K}, {B} batches x 10000 rows/step"
                               + (", producer record index (psx_apply_indexed)" if indexed else "")
                               + (", decode overlapped with the previous call's apply (PSX_PIPELINE_ALL)"
                                  if pipeline else ""),
                   "updates_per_step": nupd, "stream_bytes_per_step": stream_bytes},
        "decode": decode, "decode_variant": decode_variant, "walk_calls": walk_calls,
        "ordered_apply_ms_per_step": round(apply_ms / max(apply_n, 1), 4),
        "kernel_ms_per_step_breakdown_pass": {k: round(v[0] / max(v[1], 1), 4) for k, v in kern.items()},
        "latency_model": model,
        "roofline": roof,
        "cpu_baseline": cpu}


def run_c3(args):
    m = c3_measure(args, args.indexed, args.steps, args.warmup, args.cpu_seconds)
    p = c3_measure(args, args.indexed, args.steps, args.warmup, 0.0, pipeline=True)
    m["pipelined"] = {k: p[k] for k in ("value", "unit", "ms_per_step", "ordered_apply_ms_per_step", "decode",
                                        "host_enqueue_ms_per_step")}
    m["pipelined"]["what"] = p["config"]["workload"]
    print(json.dumps(m), flush=True)


def progress(msg, rank=0):
    """A progress line on stderr (long runs must keep writing: the GPU box takes 3 silent
    minutes for a hang)."""
    if rank == 0:
        print(f"[bench {time.strftime('%H:%M:%S')}] {msg}", file=sys.stderr, flush=True)



# ---- GPU telemetry (attribute the box-to-box spread of the headline) -----
# Read-only amdsmi queries: clocks, power, temperatures and throttle state of the GPU this
# rank drives, matched to torch's device by PCI address.  Never inside a timed region: a
# snapshot before and after it, and samples from a background thread during an untimed
# repeat of the same steps.
SMI_KEYS = ("current_gfxclk", "average_gfxclk_frequency", "current_uclk", "average_uclk_frequency",
            "current_socket_power", "average_socket_power", "temperature_hotspot", "temperature_mem",
            "temperature_edge", "gfx_activity", "umc_activity", "mem_activity", "throttle_status",
            "indep_throttle_status", "current_gfxclks", "current_socclks", "current_vclk0s")
SMI_VIOLATION_KEYS = ("active_prochot_thrm", "active_ppt_pwr", "active_socket_thrm", "active_vr_thrm",
                      "active_hbm_thrm", "per_prochot_thrm", "per_ppt_pwr", "per_socket_thrm", "per_vr_thrm",
                      "per_hbm_thrm", "acc_counter")


def _smi_handle(local):
    import amdsmi
    import torch
    amdsmi.amdsmi_init()
    hs = amdsmi.amdsmi_get_processor_handles()
    p = torch.cuda.get_device_properties(local)
    want = (getattr(p, "pci_domain_id", None), getattr(p, "pci_bus_id", None), getattr(p, "pci_device_id", None))
    for h in hs:
        try:
            dom, bus, rest = amdsmi.amdsmi_get_gpu_device_bdf(h).split(":")
            if (int(dom, 16), int(bus, 16), int(rest.split(".")[0], 16)) == want:
                return h
        except Exception:   # noqa: BLE001
            continue
    return hs[0] if len(hs) == 1 else None


def _smi_clean(v):
    if isinstance(v, (list, tuple)):
        vals = [x for x in v if isinstance(x, (int, float)) and x not in (0xFFFF, 0xFFFFFFFF)]
        return {"min": min(vals), "max": max(vals), "n": len(vals)} if vals else None
    if isinstance(v, (int, float)) and v not in (0xFFFF, 0xFFFFFFFF, 0xFFFFFFFFFFFFFFFF):
        return v
    return None


def smi_snapshot(h):
    import amdsmi
    out = {}
    try:
        m = amdsmi.amdsmi_get_gpu_metrics_info(h)
        for k in SMI_KEYS:
            if k in m:
                out[k] = _smi_clean(m[k])
    except Exception as e:   # noqa: BLE001 - reported, never fatal
        out["metrics_error"] = repr(e)[:200]
    try:
        v = amdsmi.amdsmi_get_violation_status(h)
        out["violation"] = {k: _smi_clean(v[k]) for k in SMI_VIOLATION_KEYS if k in v}
    except Exception as e:   # noqa: BLE001
        out["violation_error"] = repr(e)[:200]
    return out


class SmiSampler:
    """Samples smi_snapshot's metrics every `period` s on a thread until stop()."""

    def __init__(self, h, period=0.002):
        import threading
        self.h, self.period, self.samples = h, period, []
        self._stop = threading.Event()
        self._t = threading.Thread(target=self._run, daemon=True)

    def _run(self):
        import amdsmi
        while not self._stop.is_set():
            try:
                m = amdsmi.amdsmi_get_gpu_metrics_info(self.h)
                self.samples.append({k: _smi_clean(m.get(k)) for k in
                                     ("current_gfxclk", "current_uclk", "current_socket_power",
                                      "temperature_hotspot", "temperature_mem", "throttle_status",
                                      "current_gfxclks")})
            except Exception:   # noqa: BLE001
                pass
            time.sleep(self.period)

    def start(self):
        self._t.start()
        return self

    def stop(self):
        self._stop.set()
        self._t.join()
        out = {"samples": len(self.samples)}
        for k in ("current_gfxclk", "current_uclk", "current_socket_power", "temperature_hotspot",
                  "temperature_mem", "throttle_status"):
            xs = sorted(x[k] for x in self.samples if isinstance(x.get(k), (int, float)))
            if xs:
                out[k] = {"min": xs[0], "median": xs[len(xs) // 2], "max": xs[-1]}
        xcd = [x["current_gfxclks"] for x in self.samples if isinstance(x.get("current_gfxclks"), dict)]
        if xcd:
            out["current_gfxclks_per_xcc"] = {"min": min(d["min"] for d in xcd), "max": max(d["max"] for d in xcd)}
        return out


def ms_spread(ms):
    xs = sorted(ms)
    if not xs:
        return None
    return {"min": round(xs[0], 4), "median": round(xs[len(xs) // 2], 4), "max": round(xs[-1], 4), "n": len(xs)}

C4_CHUNK_BYTES = (1 << 31) - 4   # a worker batch travels as Appendix-A messages of < 2 GiB (the
                                 # reference reader's int32 cursor, serialized_oplog_reader.hpp:137)


def _gen(dev, *key):
    import torch
    h = 0
    for k in key:
        h = (h * 1000003 + int(k)) % (1 << 62)
    return torch.Generator(device=dev).manual_seed(h)


def batch_perm(seed, w, rows_total, dev):
    """Worker w's batch order: every table row once, in a random order."""
    import torch
    return torch.randperm(rows_total, generator=_gen(dev, seed, 1, w), device=dev).to(torch.int32)


def batch_updates(seed, w, c, n, cap, dev):
    """The N(0, 0.01) f32 updates of worker w's chunk c (n records), from their own seed."""
    import torch
    return torch.randn(n, cap, generator=_gen(dev, seed, 2, w, c), device=dev) * 0.01


def shard_init(seed, o, shard, cap, dev):
    """Owner o's initial rows, N(0, 0.1) (matrixfact_split.cpp:234-235)."""
    import torch
    return torch.randn(shard, cap, generator=_gen(dev, seed, 3, o), device=dev) * 0.1


def batch_chunks(seed, w, rows_total, cap, dev, max_bytes):
    """Worker w's batch as Appendix-A messages of at most max_bytes each: records in the
    batch order, rpc records per message (the last takes the rest)."""
    from parameter_server_amd import wire
    rpc = (max_bytes - 20) // (4 + 4 * cap)
    perm = batch_perm(seed, w, rows_total, dev)
    chunks = []
    for c, st in enumerate(range(0, rows_total, rpc)):
        rows = perm[st:st + rpc]
        chunks.append(wire.dense_stream_torch(1, rows, batch_updates(seed, w, c, rows.numel(), cap, dev)))
    return chunks, rpc


def expected_shard(seed, world, o, bounds, cap, rpc, rounds, dev):
    """Owner o's rows after `rounds` steps, recomputed from the seeds alone (independent of
    every byte the split and the exchange moved): its initial rows, then per step, per chunk
    round c, per worker w in rank order — the order the owner's fused calls apply them in —
    w's chunk-c records that fall in [bounds[o], bounds[o+1]) added in place (one f32 add per
    element, as Server::ApplyOpLogUpdateVersion, server.cpp:154-178)."""
    lo, hi = bounds[o], bounds[o + 1]
    rows_total = bounds[-1]
    exp = shard_init(seed, o, hi - lo, cap, dev)
    perms = [batch_perm(seed, w, rows_total, dev) for w in range(world)]
    nch = (rows_total + rpc - 1) // rpc
    for _ in range(rounds):
        for c in range(nch):
            for w in range(world):
                rows = perms[w][c * rpc:(c + 1) * rpc]
                m = (rows >= lo) & (rows < hi)
                if not bool(m.any()):
                    continue
                upd = batch_updates(seed, w, c, rows.numel(), cap, dev)
                idx = (rows[m] - lo).long()
                exp[idx] += upd[m]
                del upd
    return exp


class CpuShardExchange:
    """Stand-in of parameter_server_amd.exchange.ShardExchange for the gloo CPU harness
    (`--selftest-exchange`): the same chunk rounds, the split by owner, the all-to-all (gloo)
    and the in-order apply done with torch on the CPU.  Not a product path: it lets the
    orchestration, the routing and the parity check of exchange_measure run on the CPU."""

    reverse = False   # --selftest-reverse: apply the sources in reverse rank order (parity must catch it)

    def __init__(self, init, bounds, rank, world):
        self.table, self.bounds, self.rank, self.world = init.clone(), bounds, rank, world
        self.chunks = 0
        self.sent_bytes = self.recv_bytes = 0
        self.peer_sent, self.peer_recv = [0] * world, [0] * world
        self.split_s = self.wait_s = self.sync_s = self.x_ms = 0.0

    def reset_counters(self):
        self.__init__(self.table, self.bounds, self.rank, self.world)

    def _split(self, msg):
        import torch
        recs = msg[20:].view(torch.int32).view(-1, 1 + self.table.shape[1])
        own = torch.bucketize(recs[:, 0].long(), torch.tensor(self.bounds[1:-1]), right=True)
        parts, sizes = [], []
        for o in range(self.world):
            sub = recs[own == o]
            if sub.shape[0] == 0:
                sizes.append(0)
                continue
            hdr = torch.tensor([1, 1, 4, 0, sub.shape[0]], dtype=torch.int32)
            parts.append(torch.cat([hdr, sub.reshape(-1)]).view(torch.uint8))
            sizes.append(parts[-1].numel())
        return (torch.cat(parts) if parts else torch.zeros(0, dtype=torch.uint8)), sizes

    def run(self, chunks, log=None):
        import torch
        from parameter_server_amd.exchange import alltoall_streams
        lo = self.bounds[self.rank]
        for msg in chunks:
            send, sizes = self._split(msg)
            recv, rs = alltoall_streams(send, sizes)
            offs = [sum(rs[:w]) for w in range(self.world)]
            for w in (reversed(range(self.world)) if self.reverse else range(self.world)):
                if rs[w]:
                    sub = recv[offs[w]:offs[w] + rs[w]]
                    n = int(sub[16:20].view(torch.int32).item())
                    recs = sub[20:].view(torch.int32).view(n, -1)
                    idx = (recs[:, 0] - lo).long()
                    self.table[idx] += recs[:, 1:].view(torch.float32)
            self.chunks += 1
            self.sent_bytes += sum(sizes)
            self.recv_bytes += sum(rs)
            for p in range(self.world):
                if p != self.rank:      # what crosses (a rank's own part stays)
                    self.peer_sent[p] += int(sizes[p])
                    self.peer_recv[p] += int(rs[p])

    def comm_info(self):
        import torch.distributed as dist
        return {"backend": "gloo (CPU stand-in)", "nranks": dist.get_world_size() if dist.is_initialized() else 1,
                "rank": dist.get_rank() if dist.is_initialized() else 0, "device": None, "rccl_version": None,
                "librccl": None}

    def peer_bytes(self, reset=False):
        out = (list(self.peer_sent), list(self.peer_recv))
        if reset:
            self.peer_sent, self.peer_recv = [0] * self.world, [0] * self.world
        return out

    def read_table(self):
        return self.table

    def close(self):
        pass


class GlooExchange:
    """Test transport with the interface ShardExchange drives (world, rank, sizes_async,
    streams_v, close) over the gloo process group on host copies, so that several ranks can
    share one GPU (RCCL cannot put two ranks on one device).  Synchronous: each call waits for
    the device (the split that filled `send`), crosses on the host and copies the received
    bytes into `recv` before returning.  Not a product path: it lets tests/test_split_gpu.py
    run ShardExchange's multi-rank routing (displacements, the own sub-stream applied from the
    send slot, per-source versions) with the real split and apply on a one-GPU box."""

    def __init__(self):
        import torch.distributed as dist
        self.world, self.rank = dist.get_world_size(), dist.get_rank()
        self.peer_sent, self.peer_recv = [0] * self.world, [0] * self.world

    def info(self):
        return {"backend": "gloo (host copies; test transport)", "nranks": self.world, "rank": self.rank,
                "device": None, "rccl_version": None, "librccl": None}

    def peer_bytes(self, reset=False):
        out = (list(self.peer_sent), list(self.peer_recv))
        if reset:
            self.peer_sent, self.peer_recv = [0] * self.world, [0] * self.world
        return out

    def sizes_async(self, send_sizes, recv_sizes, stream):
        import torch
        import torch.distributed as dist
        rs = torch.empty(self.world, dtype=torch.int64)
        dist.all_to_all_single(rs, torch.tensor([int(x) for x in send_sizes], dtype=torch.int64))
        recv_sizes[:self.world].copy_(rs)

    def streams_v(self, send, send_sizes, send_displs, recv, recv_sizes, recv_displs, stream):
        import torch
        import torch.distributed as dist
        torch.cuda.synchronize(send.device)
        parts = [send[int(o):int(o) + int(z)] for o, z in zip(send_displs, send_sizes)]
        out = torch.cat(parts).cpu() if parts else torch.zeros(0, dtype=torch.uint8)
        got = torch.empty(sum(int(z) for z in recv_sizes), dtype=torch.uint8)
        dist.all_to_all_single(got, out, [int(z) for z in recv_sizes], [int(z) for z in send_sizes])
        for o, z, st in zip(recv_displs, recv_sizes, [sum(int(z) for z in recv_sizes[:p]) for p in range(self.world)]):
            if int(z):
                recv[int(o):int(o) + int(z)].copy_(got[st:st + int(z)])
        torch.cuda.synchronize(send.device)
        for p in range(self.world):
            self.peer_sent[p] += int(send_sizes[p])
            self.peer_recv[p] += int(recv_sizes[p])

    def close(self):
        pass


def exchange_measure(rows_total, cap, steps, warmup, world, rank, local, seed=4242, backend="psx",
                     max_bytes=C4_CHUNK_BYTES, split_single=False):
    """The exchange-bearing step, self-checked.  A dense f32 table of
    rows_total x cap, row-range sharded over the ranks (initial rows N(0, 0.1)).  Every rank is
    one worker whose batch covers every row once in a random order (updates N(0, 0.01)),
    carried as Appendix-A messages of < 2 GiB.  Per step each rank pushes its batch through
    ShardExchange (psx): per chunk, device split per owner (psx_split_stream_formats), sizes
    and bytes over libpsx's RCCL communicator, the owner's fused in-order apply — chunk k's
    exchange beside chunk k-1's apply.  After the timed steps every owner compares its shard
    bit for bit with expected_shard(), recomputed from the seeds (never from the delivered
    bytes): `parity` is "bit-exact" or the count of differing values over all ranks.
    backend "cpu": the same orchestration with CpuShardExchange under gloo (CPU tests);
    "psx-gloo": ShardExchange on the device with the bytes over gloo (GlooExchange; tests).
    One rank applies its chunks directly (nothing routes) unless split_single."""
    import torch
    import torch.distributed as dist
    cpu = backend == "cpu"
    red_dev = "cpu" if backend != "psx" else None      # gloo reduces host tensors
    dev = torch.device("cpu") if cpu else torch.device("cuda", local)
    assert rows_total % world == 0, "row-range shards of equal size"
    shard = rows_total // world
    bounds = [w * shard for w in range(world + 1)]
    lo = bounds[rank]
    t_gen = time.perf_counter()
    progress(f"exchange_measure {rows_total} x {cap}, world {world}: generating", rank)
    chunks, rpc = batch_chunks(seed, rank, rows_total, cap, dev, max_bytes)
    init = shard_init(seed, rank, shard, cap, dev)
    bgs = [100 + w for w in range(world)]
    xc = srv = None
    if cpu:
        ex = CpuShardExchange(init, bounds, rank, world)
    else:
        import parameter_server_amd as psa
        from parameter_server_amd.exchange import Exchange, ShardExchange
        srv = psa.Server(device=local, server_id=1 + rank, bg_ids=bgs)
        info = psa.TableInfo(row_kind=psa.ROW_DENSE, dtype=psa.F32, row_capacity=cap, row_offset=lo, max_rows=shard)
        srv.CreateTable(1, info)
        srv.load_rows(1, lo, None, on_device_ptr=init.data_ptr(), num_rows=shard)
        torch.cuda.synchronize()
        xc = GlooExchange() if backend == "psx-gloo" else Exchange(local)
        ex = ShardExchange(srv, 1, info, bounds, bgs, xc, local, split_single=split_single)
    del init
    if not cpu:
        torch.cuda.synchronize()
        torch.cuda.empty_cache()
    gen_s = time.perf_counter() - t_gen

    def sync():
        if not cpu:
            torch.cuda.synchronize()

    progress(f"{len(chunks)} chunks of {rpc} records; warmup", rank)
    verbose = (lambda m: progress(m, rank)) if os.environ.get("PSX_BENCH_VERBOSE") else None
    if verbose and os.environ.get("PSX_BENCH_STACK_AFTER"):
        import faulthandler        # diagnosis: where the host waits if a step never finishes
        faulthandler.dump_traceback_later(float(os.environ["PSX_BENCH_STACK_AFTER"]), exit=True)
    for _ in range(warmup):
        ex.run(chunks, log=verbose)
        sync()
        progress("warmup step done", rank)
    ex.reset_counters()
    xport = ex if cpu else xc            # whatever carries the bytes: libpsx's RCCL comm, or gloo
    xport.peer_bytes(reset=True)
    if srv is not None:
        srv.timing(2)
        srv.timing_reset()
    if world > 1:
        dist.barrier()
    sync()
    t0 = time.perf_counter()
    for _ in range(steps):
        ex.run(chunks)
    sync()
    if world > 1:
        dist.barrier()
    el = time.perf_counter() - t0
    comm = comm_view(xport, world, steps)
    progress(f"{steps} timed steps in {el:.3f} s; checking parity", rank)
    apply_ms, apply_n = srv.timing_read("dense_apply") if srv is not None else (0.0, 0)
    hbm_used = None
    if not cpu:
        free, total = torch.cuda.mem_get_info(local)
        hbm_used = total - free
    msg_bytes = sum(c.numel() for c in chunks)
    nchunks = len(chunks)
    del chunks
    # parity: the owner's shard against the seeds
    t_chk = time.perf_counter()
    if srv is not None:
        got = torch.empty(shard, cap, dtype=torch.float32, device=dev)
        srv.read_rows_device(1, lo, shard, got)
    else:
        got = ex.read_table()
    exp = expected_shard(seed, world, rank, bounds, cap, rpc, warmup + steps, dev)
    ndiff = int((got.view(torch.int32) != exp.view(torch.int32)).sum().item())
    del got, exp
    chk_s = time.perf_counter() - t_chk
    st = dict(split_s=ex.split_s, wait_s=ex.wait_s, sync_s=ex.sync_s, x_ms=ex.x_ms, chunks=ex.chunks,
              sent=ex.sent_bytes, recv=ex.recv_bytes)
    ex.close()
    if srv is not None:
        srv.close()
    if xc is not None:
        xc.close()
    if not cpu:
        torch.cuda.empty_cache()
    vals = [el, st["split_s"], st["wait_s"], st["sync_s"], st["x_ms"], apply_ms / max(apply_n, 1), gen_s, chk_s,
            float(hbm_used or 0)]
    sums = [float(ndiff), float(st["recv"])]
    if world > 1:
        t = torch.tensor(vals, dtype=torch.float64, device=red_dev or dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        vals = t.tolist()
        t = torch.tensor(sums, dtype=torch.float64, device=red_dev or dev)
        dist.all_reduce(t, op=dist.ReduceOp.SUM)
        sums = t.tolist()
    el, split_s, wait_s, sync_s, x_ms, apply_ms, gen_s, chk_s, hbm_used = vals
    ndiff, recv_all = int(sums[0]), sums[1]
    per_step = el / steps
    # algorithmic bytes per step, all owners: the received records once + every row read and
    # written once (SURVEY §8(d) C4 "reduced payload + 2 x RMW", with the payload the N
    # workers' records — the all-to-all form)
    apply_bytes = recv_all / steps + 2.0 * rows_total * cap * 4
    xbytes = msg_bytes * (world - 1) / world          # per rank per step, crossing xGMI
    if comm.get("crossed_bytes_per_step_max_rank"):
        xbytes = comm["crossed_bytes_per_step_max_rank"]   # measured by the transport itself
    return {
        "value": round(apply_bytes / per_step / 1e9, 2), "unit": "GB/s (algorithmic apply bytes, all ranks)",
        "n_gpus": world, "steps": steps, "warmup": warmup,
        "ms_per_step": round(per_step * 1e3, 3),
        "parity": "bit-exact" if ndiff == 0 else f"{ndiff} values differ",
        "parity_check": "every owner's shard vs an in-order f32 sum recomputed from the seeds "
                        "(expected_shard), bit for bit, after warmup + steps rounds",
        "chunks_per_step": nchunks, "records_per_chunk": rpc,
        "split_host_ms_per_step": round(split_s / steps * 1e3, 3),
        "exchange_wait_ms_per_step": round(wait_s / steps * 1e3, 3),
        "apply_wait_ms_per_step": round(sync_s / steps * 1e3, 3),
        "exchange_kernel_ms_per_step": round(x_ms / steps, 3) if not cpu else None,
        # nccl-tests all-to-all convention: algbw = bytes a rank sends / time, busbw = the
        # share that crosses the links, (n-1)/n of it
        "exchange_algbw_GBps": round(msg_bytes / (x_ms / steps / 1e3) / 1e9, 2) if x_ms > 0 else None,
        "exchange_busbw_GBps": round(xbytes / (x_ms / steps / 1e3) / 1e9, 2) if x_ms > 0 and world > 1 else None,
        "exchange_note": None if world > 1 else
                         "one rank: its own sub-stream never crosses (applied where it lies), so no exchange "
                         "bandwidth exists to report; comm shows the communicator libpsx built",
        "comm": comm,
        "apply_kernel_ms_per_chunk": round(apply_ms, 3) if apply_ms else None,
        "hbm_used_GB_max_rank": round(hbm_used / 1e9, 2) if hbm_used else None,
        "setup_s": round(gen_s, 2), "check_s": round(chk_s, 2),
        "config": {"workload": f"{rows_total} rows x {cap} f32, row-range shards x{world}",
                   "shard_rows": shard, "batch_bytes_per_rank": msg_bytes,
                   "parallelism": f"{world} shards; per chunk: device split per owner (psx_split_stream_formats), "
                                  f"libpsx RCCL all-to-all-v (psx_exchange_sizes_async / psx_exchange_streams), "
                                  f"fused in-order apply; chunk k's exchange beside chunk k-1's apply"
                                  if not cpu and (world > 1 or split_single) else
                                  "one rank: each chunk applied as it is (nothing routes)" if not cpu else
                                  f"{world} shards over gloo (CPU stand-in)"},
    }


def comm_view(xport, world, steps):
    """What each rank's transport itself reports, gathered to every rank: for
    libpsx's RCCL communicator, psx_comm_info (ncclCommCount / ncclCommUserRank /
    ncclCommCuDevice / ncclGetVersion and the librccl the process loaded) and
    psx_comm_peer_bytes (bytes enqueued to / from each peer over the timed steps).  A launch
    whose ranks did not all build one communicator of `world` ranks says so here
    (`all_ranks_see_world` false), whatever torch's world size is."""
    import torch.distributed as dist
    info = xport.info() if hasattr(xport, "info") else xport.comm_info()
    sent, recv = xport.peer_bytes()
    mine = dict(info)
    mine["sent_bytes_per_peer"] = sent
    mine["recv_bytes_per_peer"] = recv
    ranks = [None] * world
    if world > 1:
        dist.all_gather_object(ranks, mine)
    else:
        ranks = [mine]
    crossed = [sum(r["sent_bytes_per_peer"]) - r["sent_bytes_per_peer"][i] for i, r in enumerate(ranks)]
    return {
        "backend": ranks[0].get("backend", "rccl (libpsx psx_comm: grouped ncclSend/ncclRecv)"),
        "ranks": ranks,
        "all_ranks_see_world": all(r["nranks"] == world and r["rank"] == i for i, r in enumerate(ranks)),
        "distinct_devices": len({r["device"] for r in ranks}) if ranks[0].get("device") is not None else None,
        "crossed_bytes_per_step_max_rank": max(crossed) / steps if steps else None,
        "crossed_bytes_per_step_all_ranks": sum(crossed) / steps if steps else None,
    }


def rank_view(world, rank, local):
    """Every rank's own identity, gathered (all ranks call it): its torch rank/world, the
    device it drives (PCI bus id: distinct ids mean distinct GPUs) and the RCCL version
    torch's process group links.  For paths with no data-path collective (C5's row-range
    shards, the headline's pre-split batches) this is the evidence of how many GPUs ran."""
    import torch
    import torch.distributed as dist
    p = torch.cuda.get_device_properties(local)
    try:
        nv = ".".join(str(x) for x in torch.cuda.nccl.version())
    except Exception:   # noqa: BLE001 - reported, not fatal
        nv = None
    mine = {"rank": rank, "world": world, "local_device": local,
            "pci": f"{getattr(p, 'pci_domain_id', 0):04x}:{getattr(p, 'pci_bus_id', 0):02x}:"
                   f"{getattr(p, 'pci_device_id', 0):02x}",
            "uuid": str(getattr(p, "uuid", "")), "name": p.name, "torch_rccl": nv}
    out = [None] * world
    if world > 1:
        dist.all_gather_object(out, mine)
    else:
        out = [mine]
    return {"ranks": out, "distinct_gpus": len({(r["pci"], r["uuid"]) for r in out})}


def run_c4(args):
    """a dense f32 gradient table of c4_rows x 1024, row-range sharded
    over the ranks; every rank's batch spans every shard (exchange_measure).  N = 1 is the
    same pipeline with a one-rank (self) exchange."""
    import torch
    import torch.distributed as dist
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    if world > 1:
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    m = exchange_measure(args.c4_rows, 1024, args.steps, args.warmup, world, rank, local)
    if rank == 0:
        m["config"]["workload"] = "C4: " + m["config"]["workload"]
        line = {"metric": "C4 dense gradient apply with all-to-all exchange"}
        line.update(m)
        line.update({"higher_is_better": True, "scaling": "strong", "dtype": "f32",
                     "data": "synthetic (GPU-generated N(0,0.01) gradients, full coverage, random row order)"})
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


def selftest_exchange(args):
    """exchange_measure's orchestration and parity check under gloo on the CPU (world 2 in
    tests/test_bench_launch.py), with CpuShardExchange in place of the device path and
    messages small enough that a batch takes several chunks."""
    import torch.distributed as dist
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    if world > 1:
        dist.init_process_group("gloo")
    CpuShardExchange.reverse = args.selftest_reverse
    if args.selftest_device:
        import torch
        torch.cuda.set_device(0)
        # rows of 64 f32, 7 chunks a batch of which the last is short
        m = exchange_measure(4096 * world, 64, args.steps, args.warmup, world, rank, 0, backend="psx-gloo",
                             max_bytes=20 + 260 * 600)
    else:
        m = exchange_measure(4096 * world, 16, args.steps, args.warmup, world, rank, 0, backend="cpu",
                             max_bytes=20 + 68 * 1000)
    if rank == 0:
        m["metric"] = "selftest-exchange"
        print(json.dumps(m), flush=True)
    if world > 1:
        dist.destroy_process_group()


def run_c4shard(args):
    """SURVEY §8(d) C4, one GPU's shard: the 10M x 1024 f32 table row-range sharded over 8
    GPUs gives each GPU 1.25M rows; per step its owner receives one full-coverage message
    from each of the 8 workers (their per-owner sub-streams, rows in random order: 5.1 GB
    each, 41 GB per step), applied in one fused, order-preserving call through the
    reference-shaped psx_apply_streams_device (row ids read from the stream; each call's
    index stage beside the previous call's apply).  The 8-GPU run adds the all-to-all that
    delivers those messages (`--workload c4 --gpus 8`, driver-run).  cpu_baseline: the oracle
    on a 2^15-row shard of the same shape, extrapolated to the full shard (labelled)."""
    import torch
    import parameter_server_amd as psa
    from parameter_server_amd import wire
    W, cap = 8, 1024
    rows = args.c4_rows // W
    g = torch.Generator(device="cuda").manual_seed(4242)
    table0 = torch.randn(rows, cap, device="cuda", generator=g) * 0.1
    streams = []
    for w in range(W):
        perm = torch.randperm(rows, device="cuda", generator=g).to(torch.int32)
        upd = torch.randn(rows, cap, device="cuda", generator=g) * 0.01
        streams.append(wire.dense_stream_torch(1, perm, upd))
        del upd, perm
    torch.cuda.synchronize()
    bgs = [100 + w for w in range(W)]
    srv = psa.Server(device=0, server_id=1, bg_ids=bgs)
    srv.set_stream(torch.cuda.current_stream().cuda_stream)
    srv.set_pipeline(2)
    srv.CreateTable(1, psa.TableInfo(row_kind=psa.ROW_DENSE, dtype=psa.F32, row_capacity=cap, max_rows=rows))
    srv.load_rows(1, 0, None, on_device_ptr=table0.data_ptr(), num_rows=rows)
    del table0
    torch.cuda.empty_cache()
    ver = [0]

    def step():
        srv.apply_device([(x.data_ptr(), x.numel(), bgs[w], ver[0]) for w, x in enumerate(streams)])
        ver[0] += 1

    for _ in range(args.warmup):
        step()
    srv.sync()
    srv.timing(2)
    srv.timing_reset()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    srv.sync()
    apply_ms, apply_n = srv.timing_read("dense_apply")
    srv.timing(False)
    srv.close()
    step_bytes = sum(x.numel() for x in streams) + 2 * rows * cap * 4
    del streams
    torch.cuda.empty_cache()
    apply_s = apply_ms / max(apply_n, 1) / 1e3
    cpu = None
    if args.cpu_seconds > 0:
        cpu = cpu_baseline(args, rows=1 << 15, cap=cap)
        cpu["extrapolated_ms_per_step_full_shard"] = round(step_bytes / (cpu["value"] * 1e9) * 1e3, 1)
        cpu["sample"] = "EXTRAPOLATED from a 2^15-row shard sample: " + cpu["sample"]
    print(json.dumps({
        "metric": "C4 one GPU's shard: dense gradient apply GB/s (device-resident)",
        "value": round(step_bytes * args.steps / el / 1e9, 2), "unit": "GB/s",
        "n_gpus": 1, "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(el / args.steps * 1e3, 3),
        "higher_is_better": True, "dtype": "f32", "data": "synthetic (GPU-generated, full coverage, random order)",
        "config": {"workload": f"C4 shard: {rows} rows x {cap} f32 (10M x 1K over 8 GPUs), {W} worker messages "
                               f"per step, psx_apply_streams_device, PSX_PIPELINE_ALL",
                   "algorithmic_bytes_per_step": step_bytes},
        "roofline": {"bound": "hbm", "kernel": "dense_apply", "achieved": round(step_bytes / apply_s / 1e9, 2),
                     "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": round(step_bytes / apply_s / 1e9 / HBM_PEAK_GBS, 4),
                     "avg_launch_ms": round(apply_s * 1e3, 3)},
        "cpu_baseline": cpu}), flush=True)


def read_sweep_rate(bufs, reps=5):
    """GB/s of psx_debug_read_sweep over the device buffers `bufs` (bytes / time summed over
    all of them), or None when the hook fails."""
    from parameter_server_amd import _abi
    L = _abi.load()
    tot_b, tot_s = 0.0, 0.0
    for t in bufs:
        nb = (t.numel() * t.element_size()) // 16384 * 16384
        if nb < 16384:
            continue
        g = L.psx_debug_read_sweep(t.data_ptr(), nb, reps)
        if g <= 0:
            return None
        tot_b += nb
        tot_s += nb / (g * 1e9)
    return tot_b / tot_s / 1e9 if tot_s > 0 else None


def run_seam(args, host, rows, cap, bgs, base, local):
    """The drop-in seam as INTEGRATION.md binds it: C2's 8 messages from page-locked host
    memory (worker socket buffers), one psx_apply_stream call each (Server::
    ApplyOpLogUpdateVersion, one host message per call, server_thread.cpp:241-243), into a
    fresh context.  Each call returns once its bytes are in HBM; message k's apply runs
    beside message k+1's copy.  `value` = message bytes per second (the caller's bytes
    crossing PCIe, applied); also timed from pageable copies of the same messages."""
    import torch
    import parameter_server_amd as psa
    srv = psa.Server(device=local, server_id=99, bg_ids=bgs)
    srv.CreateTable(1, psa.TableInfo(row_kind=psa.ROW_DENSE, dtype=psa.F32, row_capacity=cap,
                                     row_offset=base, max_rows=rows))
    ver = [0]

    def step(msgs):
        for b, m in enumerate(msgs):
            srv.ApplyOpLogUpdateVersion(m, m.size, bgs[b], ver[0])
        ver[0] += 1

    pinned = [h.numpy() for h in host]
    step(pinned)
    srv.sync()
    n = max(4, args.steps // 2)
    t0 = time.perf_counter()
    for _ in range(n):
        step(pinned)
    srv.sync()
    el = time.perf_counter() - t0
    pageable = [p.copy() for p in pinned]
    step(pageable)
    srv.sync()
    t1 = time.perf_counter()
    npg = 2
    for _ in range(npg):
        step(pageable)
    srv.sync()
    el_p = time.perf_counter() - t1
    del pageable
    srv.close()
    nbytes = sum(p.size for p in pinned)
    return {"value": round(nbytes * n / el / 1e9, 2), "unit": "GB/s", "ms_per_step": round(el / n * 1e3, 3),
            "steps": n, "calls_per_step": len(pinned), "bytes_per_step": nbytes,
            "pageable_GBps": round(nbytes * npg / el_p / 1e9, 2),
            "what": "C2's 8 messages from page-locked host memory, one psx_apply_stream (ApplyOpLogUpdateVersion) "
                    "call each, settled by one psx_sync per step: message bytes per second; each call returns once "
                    "its bytes are in HBM, its apply beside the next call's copy (PSX_SEAM_ASYNC); pageable_GBps: "
                    "the same from pageable copies"}


def run_pcie(args, srv, streams, rows, cap, bgs, ver, host=None):
    """Host-resident form of C2: messages start in pinned host memory (worker socket
    buffers) and every dirty row is served back to host memory each step.

    Pipelined (the reported rate): step k+1's messages cross PCIe host-to-device on their
    own stream (into the other of two device buffer sets) while step k is applied and its
    rows cross device-to-host on a third; PCIe is full duplex, so the step costs about the
    host-to-device copy alone.  `serial` times the same work one step at a time."""
    import torch
    if host is None:
        host = [s.cpu().pin_memory() for s in streams]
    dev = [list(streams), [torch.empty_like(s) for s in streams]]
    table_host = torch.empty(rows * cap, dtype=torch.float32).pin_memory()
    table_dev = torch.empty(rows * cap, dtype=torch.float32, device="cuda")
    from parameter_server_amd import _abi
    L = _abi.load()
    first = srv.tables[1].row_offset
    cur = torch.cuda.current_stream()     # the context's stream (srv.set_stream)
    s_in, s_out = torch.cuda.Stream(), torch.cuda.Stream()
    ev_in = [torch.cuda.Event(), torch.cuda.Event()]
    ev_out = torch.cuda.Event()

    def h2d(k):
        with torch.cuda.stream(s_in):
            for h, d in zip(host, dev[k % 2]):
                d.copy_(h, non_blocking=True)
            ev_in[k % 2].record(s_in)

    def serve(k):
        cur.wait_event(ev_out)            # the previous step's rows have left table_dev
        assert L.psx_table_read_rows(srv.handle, 1, first, rows, table_dev.data_ptr(), 1) == 0
        with torch.cuda.stream(s_out):
            table_host.copy_(table_dev, non_blocking=True)
            ev_out.record(s_out)

    def apply(k):
        cur.wait_event(ev_in[k % 2])
        srv.apply_device([(d.data_ptr(), d.numel(), bgs[b], ver[0]) for b, d in enumerate(dev[k % 2])])
        ver[0] += 1

    def run(n):
        h2d(0)
        for k in range(n):
            apply(k)
            if k + 1 < n:
                h2d(k + 1)    # buffer set (k+1) % 2 was last read by apply(k-1), finished in serve(k-1)
            serve(k)          # blocks the host until apply(k) is done
        torch.cuda.synchronize()

    run(2)
    t0 = time.perf_counter()
    n = max(4, args.steps // 2)
    run(n)
    el = time.perf_counter() - t0

    def serial_step():
        h2d(0)
        apply(0)
        serve(0)
        torch.cuda.synchronize()
    serial_step()
    t1 = time.perf_counter()
    ns = 3
    for _ in range(ns):
        serial_step()
    el_s = time.perf_counter() - t1
    moved = sum(s.numel() for s in streams) + rows * cap * 4
    return {"pcie_inclusive_GBps": round(moved * n / el / 1e9, 2), "ms_per_step": round(el / n * 1e3, 3),
            "bytes_per_step": moved, "steps": n,
            "what": "pinned H2D of all messages + fused apply + D2H of every row (served back), per step; the "
                    "next step's H2D overlapped with this step's apply and D2H (two device buffer sets, "
                    "three streams), pipeline fill included",
            "serial": {"pcie_inclusive_GBps": round(moved * ns / el_s / 1e9, 2),
                       "ms_per_step": round(el_s / ns * 1e3, 3), "steps": ns}}


PCIE_PEAK_GBS = 63.0   # PCIe Gen5 x16 spec (MI355X_MICROARCH.md, chip-level parameters)


def c5_workload(rng_seed=77):
    """C5's per-clock messages (one per worker) and each client's subscriptions."""
    import numpy as np
    from parameter_server_amd import wire
    rows_d, cap, rows_s, K, B = 1 << 18, 256, 100_000, 1024, 8
    rng = np.random.RandomState(rng_seed)
    p = 1.0 / np.arange(1, rows_s + 1)
    p /= p.sum()
    parts, subs = [], []
    for b in range(B):
        ids_d = rng.permutation(rows_d)[: rows_d // 2].astype(np.int32)
        upd = rng.normal(0, 0.01, size=(ids_d.size, cap)).astype(np.float32)
        ids_s = rng.choice(rows_s, size=1250, replace=False, p=p).astype(np.int32)
        cnt = np.zeros((ids_s.size, K), np.int32)
        for r in range(ids_s.size):
            c = rng.choice(K, size=rng.randint(1, 33), replace=False)
            cnt[r, c] = rng.choice([-1, 1, 2], size=c.size)
        parts.append((ids_d, upd, ids_s, cnt))
        subs.append((ids_d, ids_s))
    msgs = [wire.pack_np([dict(table_id=1, dense_serialized=True, row_ids=a, oplogs=u),
                          dict(table_id=3, dense_serialized=False, row_ids=c, oplogs=n)]) for a, u, c, n in parts]
    return dict(rows_d=rows_d, cap=cap, rows_s=rows_s, K=K, B=B, parts=parts, msgs=msgs, subs=subs)


def c5_cpu_baseline(args, wl, seconds):
    """The oracle running C5's clocks as T server threads (rows sharded row % T,
    context.hpp:291-304; each worker's message split per server, abstract_bg_worker.cpp:
    590-649): per clock every shard applies its 8 sub-messages, advances each sender's clock
    (ClockUntil) and, when the min clock moves, serializes one push body per client from its
    subscriptions (CreateSendServerPushRowMsgs) — the same work the GPU clock does."""
    import numpy as np
    from concurrent.futures import ThreadPoolExecutor
    from oracle.oracle import OracleServer, DENSE, SORTED_MAP, F32, I32
    from parameter_server_amd import wire
    T = usable_cores()[0]
    if args.cpu_threads:
        T = min(T, args.cpu_threads)
    B, bgs = wl["B"], [100 + b for b in range(wl["B"])]

    def build(nthreads):
        shards = []
        for t in range(nthreads):
            o = OracleServer(bgs)
            o.create_table(1, DENSE, F32, wl["cap"])
            o.create_table(3, SORTED_MAP, I32, 0, oplog_dense_serialized=False)
            msgs = []
            for ids_d, upd, ids_s, cnt in wl["parts"]:
                md, ms = ids_d % nthreads == t, ids_s % nthreads == t
                msgs.append(wire.pack_np([dict(table_id=1, dense_serialized=True, row_ids=ids_d[md], oplogs=upd[md]),
                                          dict(table_id=3, dense_serialized=False, row_ids=ids_s[ms],
                                               oplogs=cnt[ms])]))
            for b, (ids_d, ids_s) in enumerate(wl["subs"]):
                for r in ids_d[ids_d % nthreads == t]:
                    o.subscribe(1, int(r), b)
                for r in ids_s[ids_s % nthreads == t]:
                    o.subscribe(3, int(r), b)
            shards.append([o, msgs, 0])
        return shards

    def clock(sh):
        o, msgs, ver = sh
        for b, m in enumerate(msgs):
            assert o.apply_stream_once(m, bgs[b], ver) == 0
        changed = 0
        for bg in bgs:
            changed = o.clock_until(bg, ver + 1) or changed
        n = sum(len(x) for x in o.serialize_push([1, 3], B)) if changed else 0
        sh[2] = ver + 1
        return n

    def timed_run(nthreads, secs):
        shards = build(nthreads)
        with ThreadPoolExecutor(nthreads) as ex:
            list(ex.map(clock, shards))      # untimed warm-up clock
            n, el = 0, 0.0
            while el < secs or n == 0:
                t0 = time.perf_counter()
                list(ex.map(clock, shards))
                el += time.perf_counter() - t0
                n += 1
        for sh in shards:
            sh[0].close()
        return n / el, n, el

    v1, n1, e1 = timed_run(1, seconds / 3)
    vt, nt, et = timed_run(T, seconds * 2 / 3) if T > 1 else (v1, n1, e1)
    return {"value": round(vt, 3), "unit": "clocks/s", "cores": T, "kind": "port", "cpu_model": cpu_model(),
            "single_thread": round(v1, 3),
            "sample": f"the same C5 workload; {T} threads (rows % {T} shards): {nt} clocks in {et:.1f} s; "
                      f"1 thread: {n1} clocks in {e1:.1f} s (oracle: single-pass apply, the reference's loop shape, "
                      f"+ ClockUntil + per-client push bodies)"}


C5_STALENESS = 4


def c5_schedule(B, clocks, staleness=C5_STALENESS, speeds=None):
    """The order in which the server receives the workers' per-clock messages under SSP
    (a discrete-event simulation in virtual time; the server is taken to be instantaneous).
    Worker w needs speeds[w] time units per clock.  Before computing clock c a worker's Get
    blocks until the server has pushed clock >= c - staleness
    (SSPPushConsistencyController::Get, ssp_push_consistency_controller.cpp:70-88); when its
    clock ends it sends the clock's message (is_clock, ClientSendOpLogMsg).  The server
    ticks the sender's clock on each message (Server::ClockUntil, server.cpp:62-79) and
    pushes when the minimum advances (server_thread.cpp:262-288), which releases gated
    workers.  Returns (arrivals, stats): arrivals lists (worker, clock, push) in arrival
    order, push = the new min clock if this message advanced it, else 0; simulated until
    every worker has sent `clocks` messages."""
    import heapq
    speeds = speeds or [1.0 + 0.25 * w for w in range(B)]   # worker 7 is 2.75x slower than worker 0
    vclock = [0] * B          # messages the server has from each worker
    pushed = 0                # the last pushed (min) clock
    blocked = []              # workers waiting in Get: (clock they want to start, worker)
    ev = [(speeds[w], w, 0) for w in range(B)]    # (finish time, worker, clock finished)
    heapq.heapify(ev)
    arrivals, n_blocked, max_lead = [], 0, 0
    while ev:
        t, w, c = heapq.heappop(ev)
        vclock[w] = c + 1
        new_min = min(vclock)
        push = new_min if new_min > pushed else 0
        max_lead = max(max_lead, max(vclock) - min(vclock))
        arrivals.append((w, c, push))
        nxt = []
        if push:
            pushed = push
            still = []
            for cw, bw in blocked:
                (nxt if pushed >= cw - staleness else still).append((cw, bw))
            blocked = still
        if c + 1 < clocks:
            if pushed >= (c + 1) - staleness:
                nxt.append((c + 1, w))
            else:
                blocked.append((c + 1, w))
                n_blocked += 1
        for cw, bw in nxt:
            heapq.heappush(ev, (t + speeds[bw], bw, cw))
    return arrivals, {"max_clock_lead": max_lead, "gate_blocks": n_blocked, "staleness": staleness,
                      "worker_speeds": speeds}


def pcie_duplex_probe(h2d_bytes, d2h_bytes, reps=3):
    """This box's PCIe: page-locked host->device alone, device->host alone, and both at once
    on two streams (GB/s, best of reps)."""
    import torch
    hsrc = torch.empty(h2d_bytes, dtype=torch.uint8).pin_memory()
    ddst = torch.empty(h2d_bytes, dtype=torch.uint8, device="cuda")
    dsrc = torch.empty(d2h_bytes, dtype=torch.uint8, device="cuda")
    hdst = torch.empty(d2h_bytes, dtype=torch.uint8).pin_memory()
    s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()

    def timed(h2d, d2h):
        best = None
        for _ in range(reps):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            if h2d:
                with torch.cuda.stream(s1):
                    ddst.copy_(hsrc, non_blocking=True)
            if d2h:
                with torch.cuda.stream(s2):
                    hdst.copy_(dsrc, non_blocking=True)
            torch.cuda.synchronize()
            el = time.perf_counter() - t0
            best = el if best is None else min(best, el)
        return best
    th, td, tb = timed(True, False), timed(False, True), timed(True, True)
    del hsrc, ddst, dsrc, hdst
    return {"h2d_GBps": round(h2d_bytes / th / 1e9, 2), "d2h_GBps": round(d2h_bytes / td / 1e9, 2),
            "both_GBps": round((h2d_bytes + d2h_bytes) / tb / 1e9, 2),
            "bytes": {"h2d": h2d_bytes, "d2h": d2h_bytes}}


def c5_host_model(wl, runs, upto, d_lo, d_hi, s_lo, s_hi):
    """Numpy recompute of one rank's C5 shard, for the line's parity field: the runs
    [0, upto) in arrival order, every message added to the rows it names in f32 (row +=
    update, one message after another: the reference's loop, server.cpp:154-178) and to the
    count matrix (the sorted-map rows' {col -> value}, SortedVectorMapStore::Inc's sums),
    with each push's dirty rows (ServerTable::AppendTableToBuffs) tracked.  Uses neither
    libpsx nor the oracle.  Returns the dense rows, the counts and the last push's dirty
    rows (dense, sparse) as shard-relative indices."""
    import numpy as np
    cap, K = wl["cap"], wl["K"]
    per = []
    for ids_d, upd, ids_s, cnt in wl["parts"]:
        md, ms = (ids_d >= d_lo) & (ids_d < d_hi), (ids_s >= s_lo) & (ids_s < s_hi)
        r, c = np.nonzero(cnt[ms])
        per.append(((ids_d[md] - d_lo).astype(np.int64), upd[md], (ids_s[ms] - s_lo).astype(np.int64)[r],
                    c.astype(np.int64), cnt[ms][r, c]))
    tab = np.zeros((d_hi - d_lo, cap), np.float32)
    cntm = np.zeros((s_hi - s_lo, K), np.int32)
    dd, ds = np.zeros(d_hi - d_lo, bool), np.zeros(s_hi - s_lo, bool)
    last = (np.zeros(0, np.int64), np.zeros(0, np.int64))
    for j in range(upto):
        group, push = runs[j]
        for w, _ in group:
            idx, upd, sr, sc, sv = per[w]
            tab[idx] += upd
            cntm[sr, sc] += sv
            dd[idx] = True
            ds[sr] = True
        if push:
            last = (np.nonzero(dd)[0], np.nonzero(ds)[0])
            dd[:] = False
            ds[:] = False
    return tab, cntm, last


def c5_parse_rows(raw, first, n, K):
    """Sorted-map records {int32 row_id; size_t size; Entry<int32>[n]} -> count matrix."""
    import numpy as np
    out = np.zeros((n, K), np.int32)
    b = np.frombuffer(raw, np.uint8)
    off = 0
    while off + 12 <= b.size:
        rid = int(b[off:off + 4].view(np.int32)[0])
        size = int(b[off + 4:off + 12].view(np.uint64)[0])
        e = b[off + 12:off + 12 + size].view(np.int32).reshape(-1, 2)
        out[rid - first, e[:, 0]] = e[:, 1]
        off += 12 + size
    return out


def c5_measure(args, world, rank, local, steps, warmup, parity=True, dump_dir=None):
    """SURVEY §8(d) C5, end to end: mixed dense + sparse tables, a continuous update stream
    under SSPPush with staleness 4, messages arriving from host memory and push bodies
    leaving to host memory.

    8 workers (= 8 clients), each sending one message per clock with both tables (a C2-like
    dense f32 table, 2^18 x 256, half the rows per worker; a C3-like SortedVectorMapRow<int32>
    table, 100K x 1024, 1250 Zipf rows per worker); each client subscribed to the rows of its
    messages (its row requests, server_thread.cpp:185-200).  The workers run at different
    speeds and the SSP gate lets the fast ones run up to 4 clocks ahead (c5_schedule), so the
    server receives later clocks' messages before it can push earlier ones.  The server
    (server_thread.cpp:224-299) takes the messages in arrival order: each run of arrivals up
    to the one that advances the min clock is copied host-to-device from page-locked memory
    (the worker socket buffers) and applied in one fused call, every sender's clock ticks
    (ClockUntil), and the push bodies (one per client, CreateSendServerPushRowMsgs,
    server.cpp:189-309) go device-to-host.  The next run's host-to-device copy overlaps this
    run's apply and push.  world > 1 (the process group already up): the tables are
    row-range sharded over the ranks; each worker's message is split per owner, as the
    reference client splits per server (abstract_bg_worker.cpp:590-649), and each rank
    serves its own shard with no collective (reductions of the timings only).
    value = pushed clocks per second (max over ranks).

    parity: after the timed region one more run to a push, untimed; then each rank's shard
    (dense rows bit for bit, sorted-map rows as {col -> value}) and that push's bodies (each
    client's row set, dense bytes, sparse values) against c5_host_model, summed over ranks.
    dump_dir: every rank also writes its shard (dense rows, sorted-map row bytes) and the
    messages it applied, in order, to dump_dir/c5_rank<r>.npz (the tests replay them through
    the oracle).  Returns the line (every rank)."""
    import numpy as np
    import torch
    import torch.distributed as dist
    import parameter_server_amd as psa
    from parameter_server_amd import wire
    wl = c5_workload()
    rows_d, cap, rows_s, K, B = wl["rows_d"], wl["cap"], wl["rows_s"], wl["K"], wl["B"]
    # this rank's row ranges and the workers' per-owner messages
    d_lo, d_hi = rank * rows_d // world, (rank + 1) * rows_d // world
    s_lo, s_hi = rank * rows_s // world, (rank + 1) * rows_s // world
    msgs, subs = [], []
    for ids_d, upd, ids_s, cnt in wl["parts"]:
        md, ms = (ids_d >= d_lo) & (ids_d < d_hi), (ids_s >= s_lo) & (ids_s < s_hi)
        msgs.append(wire.pack_np([dict(table_id=1, dense_serialized=True, row_ids=ids_d[md], oplogs=upd[md]),
                                  dict(table_id=3, dense_serialized=False, row_ids=ids_s[ms], oplogs=cnt[ms])]))
        subs.append((ids_d[md], ids_s[ms]))
    host = [torch.from_numpy(m).pin_memory() for m in msgs]           # the worker socket buffers
    mmax = max(max(m.size for m in msgs), 4)
    slots = [[torch.empty(mmax, dtype=torch.uint8, device="cuda") for _ in range(16)] for _ in range(2)]
    bgs = [100 + b for b in range(B)]
    srv = psa.Server(local, 1 + rank, bgs)
    s_apply, s_in = torch.cuda.Stream(), torch.cuda.Stream()
    srv.set_stream(s_apply.cuda_stream)
    srv.CreateTable(1, psa.TableInfo(row_kind=psa.ROW_DENSE, dtype=psa.F32, row_capacity=cap,
                                     row_offset=d_lo, max_rows=d_hi - d_lo))
    srv.CreateTable(3, psa.TableInfo(row_kind=psa.ROW_SORTED_MAP, dtype=psa.I32, row_capacity=K,
                                     oplog_dense_serialized=False, row_offset=s_lo, max_rows=s_hi - s_lo,
                                     max_entries=K))
    srv.set_num_clients(B)
    for b, (ids_d, ids_s) in enumerate(subs):
        srv.subscribe(1, ids_d, b)
        srv.subscribe(3, ids_s, b)
    W, Kc = warmup, steps
    pcie = pcie_duplex_probe(sum(m.size for m in msgs), 1 << 30)
    arrivals, gate = c5_schedule(B, W + Kc + C5_STALENESS + 4)
    # runs of arrivals: each ends with the message that advances the min clock
    runs, cur = [], []
    for w, c, push in arrivals:
        cur.append((w, c))
        if push or len(cur) == 16:        # a fused call takes <= 16 messages
            runs.append((cur, push))
            cur = []
    ver = [0] * B
    ev_in = [torch.cuda.Event(), torch.cuda.Event()]
    ev_used = [torch.cuda.Event(), torch.cuda.Event()]
    acct = {"h2d": 0, "d2h": 0, "msgs": 0, "pushes": 0, "apply_s": 0.0, "push_s": 0.0, "lead_at_push": 0}

    def h2d(j):
        if j >= len(runs):
            return
        k = j % 2
        s_in.wait_event(ev_used[k])                    # run j-2's apply has read slot set k
        with torch.cuda.stream(s_in):
            for i, (w, c) in enumerate(runs[j][0]):       # message i of the run -> slot i
                if host[w].numel():
                    slots[k][i][:host[w].numel()].copy_(host[w], non_blocking=True)
        ev_in[k].record(s_in)

    last_bodies = [None]

    def serve(j, keep=False):
        """One run: apply (fused), ClockUntil per message, push if the min clock moved."""
        k = j % 2
        group, push = runs[j]
        t0 = time.perf_counter()
        s_apply.wait_event(ev_in[k])
        call = []
        for i, (w, c) in enumerate(group):
            call.append((slots[k][i].data_ptr(), int(host[w].numel()), bgs[w], ver[w]))
            ver[w] += 1
        srv.apply_device(call)
        ev_used[k].record(s_apply)
        h2d(j + 1)                                     # the next run's copy beside this apply and push
        changed = 0
        for w, c in group:
            changed = srv.ClockUntil(bgs[w], c + 1) or changed
        t1 = time.perf_counter()
        pushed_bytes = 0
        if changed:
            bodies = srv.serialize_push(clear=True, as_bytes=keep)    # settles the apply; D2H
            pushed_bytes = sum(len(x) for x in bodies)
            if keep:
                last_bodies[0] = bodies
        else:
            srv.sync()
        t2 = time.perf_counter()
        return len(group), sum(int(host[w].numel()) for w, _ in group), pushed_bytes, bool(changed), t1 - t0, t2 - t1

    # warmup: the runs up to the W-th push
    j, pushes = 0, 0
    h2d(0)
    while j < len(runs) and pushes < W:
        pushes += runs[j][1] > 0
        serve(j)
        j += 1
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    t0 = time.perf_counter()
    done = 0
    while j < len(runs) and done < Kc:
        n, hb, db, ch, ta, tp = serve(j)
        acct["msgs"] += n
        acct["h2d"] += hb
        acct["d2h"] += db
        acct["apply_s"] += ta
        acct["push_s"] += tp
        done += runs[j][1] > 0
        j += 1
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    el = time.perf_counter() - t0
    check = None
    if parity:
        # untimed: the runs up to the next push, keeping its bodies; then the shard and the
        # bodies against the host model
        while j < len(runs):
            pushed = runs[j][1] > 0
            serve(j, keep=pushed)
            j += 1
            if pushed:
                break
        srv.sync()
        tab, cntm, (dirty_d, dirty_s) = c5_host_model(wl, runs, j, d_lo, d_hi, s_lo, s_hi)
        got_d = srv.read_rows(1, d_lo, d_hi - d_lo)
        bad_dense = int(np.sum(got_d.view(np.uint32) != tab.view(np.uint32)))
        raw_s = srv.serialize_rows(3, list(range(s_lo, s_hi)))
        got_s = c5_parse_rows(raw_s, s_lo, s_hi - s_lo, K)
        if dump_dir:
            order = np.array([wc for g, _ in runs[:j] for wc in g], np.int32).reshape(-1, 2)
            np.savez(os.path.join(dump_dir, f"c5_rank{rank}.npz"), dense=got_d,
                     sparse=np.frombuffer(raw_s, np.uint8), order=order,
                     bounds=np.array([d_lo, d_hi, s_lo, s_hi], np.int64))
        bad_sparse = int(np.sum(got_s != cntm))
        bad_push = 0
        if last_bodies[0] is None:
            bad_push = -1
        else:
            for b, body in enumerate(last_bodies[0]):
                parsed = wire.parse_push_body(body)
                sub_d = np.zeros(d_hi - d_lo, bool)
                sub_d[subs[b][0] - d_lo] = True
                sub_s = np.zeros(s_hi - s_lo, bool)
                sub_s[subs[b][1] - s_lo] = True
                want_d = sorted(int(r) for r in dirty_d if sub_d[r])
                want_s = sorted(int(r) for r in dirty_s if sub_s[r])
                rec_d, rec_s = parsed.get(1, {}), parsed.get(3, {})
                if sorted(r - d_lo for r in rec_d) != want_d or sorted(r - s_lo for r in rec_s) != want_s:
                    bad_push += 1
                    continue
                for r, payload in rec_d.items():
                    bad_push += payload != tab[r - d_lo].tobytes()
                for r, payload in rec_s.items():
                    e = np.frombuffer(payload, np.int32).reshape(-1, 2)
                    row = np.zeros(K, np.int32)
                    row[e[:, 0]] = e[:, 1]
                    bad_push += not np.array_equal(row, cntm[r - s_lo])
        check = [bad_dense, bad_sparse, bad_push]
    if world > 1:
        rdev = "cpu" if dist.get_backend() == "gloo" else "cuda"
        t = torch.tensor([el], dtype=torch.float64, device=rdev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        el = float(t.item())
        tot = torch.tensor([acct["h2d"], acct["d2h"]], dtype=torch.float64, device=rdev)
        dist.all_reduce(tot, op=dist.ReduceOp.SUM)
        h2d_all, d2h_all = (float(x) for x in tot.tolist())
        if check is not None:
            ct = torch.tensor([abs(x) for x in check], dtype=torch.int64, device=rdev)
            dist.all_reduce(ct, op=dist.ReduceOp.SUM)
            check = [int(x) for x in ct.tolist()]
    else:
        h2d_all, d2h_all = float(acct["h2d"]), float(acct["d2h"])
    srv.close()
    del slots
    torch.cuda.empty_cache()
    ms = el / max(done, 1) * 1e3
    touched_d = len(set().union(*[set(a.tolist()) for a, _ in subs]))
    dev_bytes = acct["h2d"] / max(done, 1) + 2 * touched_d * cap * 4 / 1.0
    h2d_pc, d2h_pc = acct["h2d"] / max(done, 1), acct["d2h"] / max(done, 1)
    bound_ms = (max(h2d_pc, d2h_pc) / (PCIE_PEAK_GBS * 1e9) + dev_bytes / (HBM_PEAK_GBS * 1e9)) * 1e3
    bound_serial_ms = ((h2d_pc + d2h_pc) / (PCIE_PEAK_GBS * 1e9) + dev_bytes / (HBM_PEAK_GBS * 1e9)) * 1e3
    cpu = c5_cpu_baseline(args, wl, min(args.cpu_seconds, 12.0)) if args.cpu_seconds > 0 and world == 1 else None
    par = None
    if check is not None:
        par = {"result": "bit-exact" if not any(check) else "MISMATCH",
               "dense_values_differing": check[0], "sparse_values_differing": check[1],
               "push_records_differing": check[2],
               "what": "every rank after the timed region and one more run to a push: its dense shard bit for bit "
                       "and its sorted-map shard as {col -> value} against a numpy replay of the same arrival-ordered "
                       "messages (f32 row += update per message; integer sums), and that push's bodies (each "
                       "client's dirty subscribed rows, dense bytes, sparse values); counts summed over ranks"}
    return {
        "metric": "C5 mixed dense+sparse clocks under SSPPush, end to end (H2D of the workers' messages, apply, "
                  "ClockUntil, per-client push bodies D2H)",
        "value": round(done / el, 2), "unit": "clocks/s",
        "ms_per_clock": round(ms, 3),
        "n_gpus": world, "steps": done, "warmup": W, "higher_is_better": True,
        "parity": par,
        "h2d_bytes_per_clock_all_ranks": int(h2d_all / max(done, 1)),
        "d2h_bytes_per_clock_all_ranks": int(d2h_all / max(done, 1)),
        "pcie_GBps_per_rank": {"h2d": round(h2d_pc / (ms / 1e3) / 1e9, 2), "d2h": round(d2h_pc / (ms / 1e3) / 1e9, 2)},
        "messages_per_clock": round(acct["msgs"] / max(done, 1), 2),
        "apply_and_clock_ms_per_clock": round(acct["apply_s"] / max(done, 1) * 1e3, 3),
        "push_ms_per_clock": round(acct["push_s"] / max(done, 1) * 1e3, 3),
        "ssp_gate": dict(gate, what="c5_schedule: worker w takes 1 + 0.25 w time units per clock; Get blocks "
                                    "until pushed clock >= clock - staleness; the server applies messages in "
                                    "arrival order, so fast workers' later clocks are applied before the push "
                                    "of earlier ones"),
        "pcie_probe": dict(pcie, note="the same copies through torch on two streams, alone and at once; "
                                      "issued this way the two directions did not overlap (both_GBps ~ one "
                                      "direction), while C5's own copies (torch H2D + libpsx D2H) move "
                                      "pcie_GBps_per_rank h2d + d2h together"),
        "bound": {"ms_per_clock": round(bound_ms, 3), "frac": round(bound_ms / ms, 3),
                  "serial_ms_per_clock": round(bound_serial_ms, 3),
                  "what": "per rank: max(H2D, D2H) bytes at the PCIe Gen5 x16 spec (63 GB/s per direction, "
                          "full duplex) + the device bytes (messages + dense row read/write) at 8 TB/s; "
                          "serial_ms: both directions in turn"},
        "dtype": "f32+int32", "data": "synthetic",
        "config": {"workload": f"C5: dense {rows_d}x{cap} f32 + sorted-map {rows_s}x{K} int32, {B} clients x 1 msg/"
                               f"clock, SSPPush, staleness {C5_STALENESS}, row-range shards x{world}",
                   "scaling": "strong (fixed workload split over the ranks)"},
        "cpu_baseline": cpu,
    }


def run_c5(args):
    """`bench.py --workload c5`: c5_measure on WORLD_SIZE ranks (one per GPU; gloo when
    --c5-gloo, e.g. several ranks sharing one GPU in the tests), rank 0 prints the line;
    --c5-dump DIR: every rank also writes its shard and its applied message order there."""
    import torch
    import torch.distributed as dist
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if args.c5_gloo:   # ranks may share a GPU (the tests' one-GPU box)
        local %= max(1, torch.cuda.device_count())
    torch.cuda.set_device(local)
    if world > 1:
        if args.c5_gloo:
            dist.init_process_group("gloo")
        else:
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    line = c5_measure(args, world, rank, local, args.steps, args.warmup, dump_dir=args.c5_dump)
    if rank == 0:
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


def main():
    args = parse()
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(launch_ranks(args))
    if args.variant:
        import torch  # noqa: F401 - torch's HIP runtime first: libpsx must bind to the same one
        from parameter_server_amd import _abi
        for kv in args.variant:
            k, v = (int(x) for x in kv.split("="))
            if _abi.load().psx_debug_set_variant(k, v) < 0:
                sys.exit(f"--variant {kv}: unknown selector")
    if args.selftest_launch:
        return selftest_launch(args)
    if args.selftest_exchange:
        return selftest_exchange(args)
    if args.workload == "c5":
        return run_c5(args)
    if args.workload == "c3":
        return run_c3(args)
    if args.workload == "c4":
        return run_c4(args)
    if args.workload == "c4shard":
        return run_c4shard(args)
    import torch
    import torch.distributed as dist
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    if world > 1:
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))

    import parameter_server_amd as psa
    from parameter_server_amd import wire

    rows, cap, B = args.rows, args.cols, args.batches
    # record-row lists only where the apply kernel uses them (v3: full coverage, no
    # importance, no AdaRevision); the other variants place records from the stream
    use_rows = not (args.walked or args.adarevision or args.importance or args.density != 1.0)
    base = rank * rows                       # this shard's first row id
    g = torch.Generator(device="cuda").manual_seed(1234 + 7919 * rank)
    table0 = torch.randn(rows, cap, device="cuda", generator=g) * 0.1
    streams = []
    nb = max(1, int(round(rows * args.density)))   # records per batch
    touched = torch.zeros(rows, dtype=torch.bool, device="cuda")
    record_rows = []   # the producer's record-row lists (psx_pack_stream_indexed's record_rows)
    for b in range(B):
        perm = torch.randperm(rows, device="cuda", generator=g)[:nb].to(torch.int32)
        touched[perm.long()] = True
        perm += base
        upd = torch.randn(nb, cap, device="cuda", generator=g) * 0.01
        if args.f16_records:
            streams.append(wire.dense_stream_torch_f16(1, perm, upd.half()))
        else:
            streams.append(wire.dense_stream_torch(1, perm, upd))
        if use_rows:
            record_rows.append(perm)
        del upd, perm
    n_touched = int(touched.sum().item())
    del touched
    torch.cuda.synchronize()

    bgs = [100 + b for b in range(B)]
    srv = psa.Server(device=local, server_id=1 + rank, bg_ids=bgs)
    srv.set_stream(torch.cuda.current_stream().cuda_stream)
    if use_rows:   # the messages are resident before the timed loop: overlap index and apply
        srv.set_pipeline(1)
    srv.CreateTable(1, psa.TableInfo(row_kind=psa.ROW_DENSE, dtype=psa.F32, row_capacity=cap,
                                     row_offset=base, max_rows=rows, accum_importance=args.importance,
                                     row_oplog_type=3 if args.f16_records else 0))
    if args.adarevision:
        srv.set_adarevision(1, init_step_size=0.1, gaussian_init=False)
    srv.load_rows(1, base, None, on_device_ptr=table0.data_ptr(), num_rows=rows)
    del table0
    torch.cuda.empty_cache()

    ver = [0]

    def step(walked=False):
        msgs = [(s.data_ptr(), s.numel(), bgs[b], ver[0]) for b, s in enumerate(streams)]
        if use_rows and not walked:
            srv.apply_indexed_rows(msgs, [r.data_ptr() for r in record_rows])
        else:
            srv.apply_device(msgs)
        ver[0] += 1

    for _ in range(args.warmup):
        step()
    srv.sync()
    torch.cuda.synchronize()

    smi = None
    try:
        smi = _smi_handle(local)
    except Exception as e:   # noqa: BLE001 - telemetry is reported, never fatal
        smi_err = repr(e)[:200]
    else:
        smi_err = None if smi is not None else "no amdsmi handle matches this device's PCI address"
    smi_before = smi_snapshot(smi) if smi is not None else None
    # Timed region: HIP events bracket only the apply launches (timing mode 2), so the
    # roofline's launch duration comes from the same steps `value` times; one event pair per
    # step on the step's stream gives the per-step spread.
    srv.timing(2)
    srv.timing_reset()
    step_ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
               for _ in range(args.steps)]
    # the events go on the stream the apply is launched on (the context's: psx_ctx_get_stream),
    # which is not torch's current stream when that is the null stream
    apply_stream = torch.cuda.ExternalStream(srv._L.psx_ctx_get_stream(srv.handle), device=local)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(args.steps):
        step_ev[i][0].record(apply_stream)
        step()
        step_ev[i][1].record(apply_stream)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    srv.sync()
    step_ms = [a.elapsed_time(b) for a, b in step_ev]
    smi_after = smi_snapshot(smi) if smi is not None else None
    # the same steps again, untimed, with a sampler thread reading clocks / power / temperature
    smi_during = None
    if smi is not None:
        sampler = SmiSampler(smi).start()
        for _ in range(max(40, args.steps)):
            step()
        torch.cuda.synchronize()
        smi_during = sampler.stop()
        srv.sync()
    apply_kernel = "ada_apply" if args.adarevision else "dense_apply"
    apply_ms, apply_n = srv.timing_read(apply_kernel)
    # Per-kernel breakdown: a separate, untimed pass with events around every kernel.
    srv.timing(1)
    srv.timing_reset()
    for _ in range(max(3, min(args.steps, 10))):
        step()
    srv.sync()
    kernels = {k: srv.timing_read(k) for k in ("decode_streams", "dense_index", "dense_verify",
                                               apply_kernel, "finish_call")}
    srv.timing(False)
    # The box's own HBM read rate (north_star: "≥70 % of single-GPU HBM read bandwidth"): a
    # read-only sweep over the resident message buffers, after the timed region.
    read_sweep = read_sweep_rate(streams)
    # The walked path (row ids read from the stream, no overlap) on the same messages, timed
    # the same way, reported beside `value`.
    walked = None
    if use_rows and not args.skip_walked:
        # the reference-shaped call at its best: the messages are resident before each call,
        # so its decode/index stage may run beside the previous call's apply
        srv.set_pipeline(2)
        for _ in range(2):
            step(walked=True)
        srv.sync()
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(args.steps):
            step(walked=True)
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        el_w = time.perf_counter() - t0
        srv.sync()
        if world > 1:
            t = torch.tensor([el_w], device="cuda", dtype=torch.float64)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            el_w = float(t.item())

    if world > 1:
        t = torch.tensor([elapsed], device="cuda", dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())

    list_bytes = sum(4 * r.numel() for r in record_rows)
    stream_bytes = sum(s.numel() for s in streams) + list_bytes
    # per GPU: streams (+ the record-row lists) + row read/write (+ accum, z, z_max read/write
    # for AdaRevision)
    step_bytes = stream_bytes + (8 if args.adarevision else 2) * n_touched * cap * 4
    total_bytes = step_bytes * args.steps * world
    value = total_bytes / elapsed / 1e9
    if walked is None and use_rows and not args.skip_walked:
        wb = step_bytes - list_bytes
        walked = {"value": round(wb * args.steps * world / el_w / 1e9, 2), "unit": "GB/s",
                  "ms_per_step": round(el_w / args.steps * 1e3, 4),
                  "what": "the same messages through psx_apply_streams_device (the reference-shaped "
                          "ApplyOpLogUpdateVersion call): row ids read from the stream (dense_index), the index "
                          "stage beside the previous call's apply (PSX_PIPELINE_ALL); algorithmic bytes without "
                          "the lists"}

    apply_avg_s = apply_ms / max(apply_n, 1) / 1e3
    achieved = step_bytes / apply_avg_s / 1e9 if apply_avg_s > 0 else None
    traffic, traffic_note = None, None
    c2_dims = ((rows, cap, B) == (1 << 20, 256, 8) and not args.importance and not args.f16_records
               and args.density == 1.0)
    pmc_json = args.pmc_json
    if args.adarevision:   # the AdaRevision kernel's own PMC passes (tools/gpu_session5.sh)
        pmc_json = os.path.join(ROOT, "profiles", "r01", "pmc_ada_apply.json")
    if c2_dims and pmc_json and os.path.exists(pmc_json):
        pmc = json.load(open(pmc_json))
        if pmc.get("kernel_signature") == kernel_signature():
            traffic = pmc.get("dense_apply_hbm_bytes_per_launch")
        else:
            traffic_note = (f"{os.path.relpath(pmc_json, ROOT)} was measured on kernel signature "
                            f"{pmc.get('kernel_signature')}, this tree is {kernel_signature()}: not reported")
    elif c2_dims:
        traffic_note = "no PMC JSON for this tree"

    def build_line(cpu):
        return {
            "metric": "row-update apply GB/s (device-resident), dense float rows"
                      + (", float16 records" if args.f16_records else "")
                      + (", AdaRevision server logic" if args.adarevision else ""),
            "value": round(value, 2),
            "unit": "GB/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(elapsed / args.steps * 1e3, 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f32",
            "data": "synthetic (GPU-generated N(0,0.1) table, N(0,0.01) updates, random row order per batch)",
            "config": {
                "workload": f"C2: DenseRow<float> table {rows} rows x {cap} cols per GPU, "
                            f"{B} worker batches (Appendix-A streams) applied per step"
                            + (f", each covering {args.density:g} of the rows" if args.density != 1.0 else ""),
                "rows_per_gpu": rows, "cols": cap, "batches_per_step": B,
                "density": args.density, "rows_touched_per_step": n_touched,
                "algorithmic_bytes_per_step_per_gpu": step_bytes,
                "parallelism": f"row-range shards x{world}, no collective",
                "importance": bool(args.importance),
                "server_table_logic": "AdaRevision" if args.adarevision else None,
                "record_format": "float16 (row_oplog_type 3)" if args.f16_records else "V[cap] (DenseRowOpLog)",
                "record_placement": ("producer record-row lists (psx_apply_indexed_rows, psx_pack_stream_indexed's "
                                     "record_rows; 4 B per record counted), every record's row id checked in the apply; "
                                     "index stage overlapped with the previous call's apply (psx_ctx_set_pipeline)"
                                     if use_rows else "row ids read from the stream (dense_index)"),
            },
            "roofline": {
                "bound": "hbm",
                "kernel": apply_kernel,
                "achieved": round(achieved, 2) if achieved else None,
                "peak": HBM_PEAK_GBS,
                "unit": "GB/s",
                "frac": round(achieved / HBM_PEAK_GBS, 4) if achieved else None,
                "traffic": traffic,
                "traffic_source": os.path.relpath(pmc_json, ROOT) if traffic else None,
                "traffic_note": traffic_note,
                "kernel_signature": kernel_signature(),
                "dram_GBps": round(traffic / apply_avg_s / 1e9, 1) if traffic and apply_avg_s > 0 else None,
                "avg_launch_ms": round(apply_avg_s * 1e3, 4),
                "read_sweep_GBps": round(read_sweep, 1) if read_sweep else None,
                "frac_of_read_sweep": round(achieved / read_sweep, 4) if achieved and read_sweep else None,
                "read_sweep_note": "this GPU's HBM read rate in the same run (psx_debug_read_sweep: 16-B "
                                   "non-temporal loads over the resident message buffers); north_star's target "
                                   "is 0.70 of single-GPU HBM read bandwidth",
            },
            "kernel_ms_per_launch_breakdown_pass": {k: round(v[0] / max(v[1], 1), 4) for k, v in kernels.items()},
            "step_ms_spread": ms_spread(step_ms),
            "telemetry": {
                "gpu": torch.cuda.get_device_properties(local).name,
                "before_timed": smi_before, "after_timed": smi_after,
                "during_untimed_repeat": smi_during,
                "error": smi_err,
                "note": "amdsmi (read-only) on this rank's GPU, matched by PCI address: a snapshot before and "
                        "after the timed region, and ~2 ms samples during an untimed repeat of the same steps "
                        "(the timed region itself runs with no sampler)",
            },
            "cpu_baseline": cpu,
        }

    # The driver runs the bare `python bench.py [--gpus N]`: on the plain C2 configuration
    # the same run also records, beside `value`, the PCIe-inclusive rate and C3 (N = 1), or
    # the exchange-bearing step over xGMI (N > 1).  None of it is inside the timed region.
    extras = args.extras and c2_dims and not args.adarevision and not args.walked
    # the messages in page-locked host memory: the PCIe-inclusive pass, the seam and the CPU
    # baseline (the full C2 messages on the host's cores) all start from them
    host = None
    if (args.pcie or extras) and world == 1:
        host = [s.cpu().pin_memory() for s in streams]
    elif world == 1 and args.cpu_seconds > 0 and c2_dims and not args.adarevision:
        host = [s.cpu() for s in streams]
    pcie = run_pcie(args, srv, streams, rows, cap, bgs, ver, host) if args.pcie or (extras and world == 1) else None
    srv.close()
    del streams, record_rows
    torch.cuda.empty_cache()
    seam = None
    if extras and world == 1:
        try:
            seam = run_seam(args, host, rows, cap, bgs, base, local)
            if pcie:
                seam["frac_of_pcie_inclusive_pipelined"] = round(seam["value"] / pcie["pcie_inclusive_GBps"], 3)
        except Exception as e:
            seam = {"error": repr(e)[:400]}
    other, exchange, c4, c5 = None, None, None, None
    if extras and world > 1:
        # The exchange extras must never cost the headline: if they have not finished within
        # EXCHANGE_TIMEOUT_S (a collective that never completes, say), rank 0 prints the line
        # without them and every rank exits with status 3, so the launcher sees the hang.
        import threading
        done = threading.Event()

        def watchdog():
            if done.wait(EXCHANGE_TIMEOUT_S):
                return
            if rank == 0:
                ln = build_line(None)
                if walked:
                    ln["walked"] = walked
                if exchange:
                    ln["exchange"] = exchange
                if c4:
                    ln["c4"] = c4
                ln["c5" if c4 else "c4" if exchange else "exchange"] = {
                    "error": f"not finished within {EXCHANGE_TIMEOUT_S} s: abandoned"}
                print(json.dumps(ln), flush=True)
            sys.stdout.flush()
            sys.stderr.flush()
            os._exit(3)
        threading.Thread(target=watchdog, daemon=True).start()
        try:
            exchange = exchange_measure(world * rows, cap, 3, 1, world, rank, local)
            exchange["what"] = ("a worker batch spanning every shard at C2's row width: per chunk, the device split "
                                "per owner, one RCCL all-to-all over xGMI, the owner's fused in-order apply; "
                                "parity against the seeds")
        except Exception as e:   # reported, never allowed to drop the headline line
            exchange = {"error": repr(e)[:400]}
        try:
            c4 = exchange_measure(args.c4_rows, 1024, 3, 1, world, rank, local)
            c4["what"] = ("SURVEY C4: the 10M x 1024 f32 table row-range sharded over the ranks, every rank's batch "
                          "spanning every shard (< 2 GiB messages), exchanged and applied per chunk; parity against "
                          "the seeds")
        except Exception as e:
            c4 = {"error": repr(e)[:400]}
        try:
            # SURVEY C5 (BASELINE configs[4], "8 MI355X"): the mixed dense + sparse SSP stream,
            # row-range sharded over the ranks, self-checked
            c5 = c5_measure(args, world, rank, local, 5, 2)
            c5.pop("metric", None)
            c5["ranks_view"] = rank_view(world, rank, local)
        except Exception as e:
            c5 = {"error": repr(e)[:400]}
        done.set()
    if extras and world == 1:
        # C3 in child processes (`bench.py --workload c3`), so its device memory and state
        # start fresh rather than where C2 and the PCIe pass left them (a C3 run right after
        # them in this process measured its apply 3x slower)
        other = {}
        cs = str(min(args.cpu_seconds, 6.0))
        for name, flags in (("C3_walked", ["--cpu-seconds", cs]),
                            ("C3_indexed", ["--indexed", "--cpu-seconds", "0"])):
            try:
                m = run_child(["--workload", "c3", "--steps", "50", "--warmup", "5"] + flags)
                other[name] = {k: m.get(k) for k in ("value", "unit", "ms_per_step", "decode",
                                                     "ordered_apply_ms_per_step",
                                                     "kernel_ms_per_step_breakdown_pass", "roofline",
                                                     "cpu_baseline", "pipelined")}
                other[name]["config"] = m["config"]["workload"]
                lm = m.get("latency_model") or {}
                other[name]["ordered_apply_frac_of_latency_bound"] = lm.get("frac_of_bound")
            except Exception as e:
                other[name] = {"error": repr(e)[:400]}
        cw, ci = other.get("C3_walked") or {}, other.get("C3_indexed") or {}
        if cw.get("cpu_baseline") and "error" not in ci:
            # the reference has no record index: its CPU apply of the indexed messages is the
            # same walk over the same bytes as the walked run's, measured once
            ci["cpu_baseline"] = dict(cw["cpu_baseline"],
                                      note="the reference has no producer record index: the same CPU apply of the "
                                           "same messages as C3_walked's cpu_baseline (measured once, in that run)")
        for name, flags in (("C4_shard_1gpu", ["--workload", "c4shard", "--steps", "5", "--warmup", "2",
                                               "--cpu-seconds", cs]),
                            ("C4_pipeline_1gpu", ["--workload", "c4", "--steps", "3", "--warmup", "1"]),
                            ("C5", ["--workload", "c5", "--steps", "10", "--warmup", "2", "--cpu-seconds", cs])):
            try:
                m = run_child(flags, timeout=400)
                m.pop("metric", None)
                other[name] = m
            except Exception as e:
                other[name] = {"error": repr(e)[:400]}
    rv = None
    if world > 1:
        try:
            rv = rank_view(world, rank, local)
        except Exception as e:   # noqa: BLE001 - reported, never allowed to drop the headline
            rv = {"error": repr(e)[:400]}
    if rank == 0:
        cpu = None
        if world == 1 and args.cpu_seconds > 0:
            full_c2 = host is not None and c2_dims and not args.adarevision
            cpu = cpu_baseline(args, host_msgs=[h.numpy() for h in host] if full_c2 else None, base=base)
        del host
        line = build_line(cpu)
        if rv:
            line["ranks_view"] = rv
        if walked:
            line["walked"] = walked
        if pcie:
            line["pcie_inclusive"] = pcie
        if seam:
            line["seam"] = seam
        if exchange:
            line["exchange"] = exchange
        if c4:
            line["c4"] = c4
        if c5:
            line["c5"] = c5
        if other:
            line["other_configs"] = other
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
