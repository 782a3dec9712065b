"""Per-record latency of the sorted-map apply (SortedVectorMapStore::Inc,
sorted_vector_map_store.hpp:305-337) on MI355X, for the C3 cost model.

One row, one wave: the row's image is first filled to n entries, then one call of 16
messages x 1 record x 64 columns is applied to it — every column an existing key
("found": FindIndex + add in place; the steady state of C3, where the same columns recur
every step) or a new key ("insert": FindIndex + LinearSearchAndMove + the shift).  The
ordered_apply launch time (HIP events, timing mode 2) / Incs is the latency of one Inc in a
dependent chain at image size n, on the kernel the product picks for that size (<= 256
entries: the 256-entry register image, else the 1,024-entry one).  ("insert": 4 records
of 64 new keys, n -> n + 256.)

Usage: python tools/probe_inc_latency.py [--out profiles/r02/c3_inc_latency.json]"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default=None)
    ap.add_argument("--reps", type=int, default=5)
    args = ap.parse_args()
    import numpy as np
    import torch
    import parameter_server_amd as psa
    from parameter_server_amd import wire
    K = 1024
    def one_call(n, nmsg, mode, rep):
        """ns of the ordered_apply launch of one call: nmsg records x 64 columns on row 0,
        whose image holds n entries (found/found_small: existing keys; insert: new keys)."""
        rng = np.random.RandomState(1000 * rep + n + 7 * nmsg)
        bgs = list(range(1, nmsg + 1))
        srv = psa.Server(0, 1, bgs + [99])
        srv.CreateTable(3, psa.TableInfo(row_kind=psa.ROW_SORTED_MAP, dtype=psa.I32, row_capacity=K,
                                         oplog_dense_serialized=False, max_rows=64, max_entries=K))
        perm = rng.permutation(K).astype(np.int32)
        have, fresh = np.sort(perm[:n]), perm[n:]
        if n:
            fill = wire.sparse_stream_np(3, 4, [(0, have, rng.randint(1, 100, size=n).astype(np.int32))])
            srv.ApplyOpLogUpdateVersion(fill.tobytes(), fill.size, 99, 0)
        msgs = []
        for b in range(nmsg):
            if mode != "insert":
                k = min(24 if mode == "found24" else 64, n)
                cols = np.sort(rng.choice(have, size=k, replace=False)).astype(np.int32)
            else:
                cols = np.sort(fresh[64 * b:64 * (b + 1)]).astype(np.int32)
            msgs.append(wire.sparse_stream_np(3, 4, [(0, cols, np.ones(cols.size, np.int32))]))
        dev = [torch.from_numpy(m).cuda() for m in msgs]
        torch.cuda.synchronize()
        srv.timing(2)
        srv.timing_reset()
        srv.apply_device([(d.data_ptr(), d.numel(), bg, 0) for d, bg in zip(dev, bgs)])
        srv.sync()
        ms, _ = srv.timing_read("ordered_apply")
        incs = sum(int(np.frombuffer(m[24:28].tobytes(), "<i4")[0]) for m in msgs)
        srv.close()
        return ms * 1e6, incs

    # Per RECORD of found keys (the sorted-map apply adds a record chunk's found keys at once,
    # found_run in psx_ordered.hip): the difference of two calls' launch times cancels the
    # launch's fixed part.  found: 16 vs 4 records of 64 existing keys (the 1,024-entry
    # image); found_small: 3 vs 1 records (n + 192 <= 256: the 256-entry image).  insert:
    # ns per new key, 4 records x 64 new keys (n -> n + 256), launch time / Incs.
    def med(n, nmsg, mode):
        return float(np.median([one_call(n, nmsg, mode, rep)[0] for rep in range(args.reps)]))
    res = {"found_rec": {}, "found_small_rec": {}, "insert": {}}
    for n in (64, 128, 192, 256, 384, 512, 768, 960):
        res["found_rec"][n] = round((med(n, 16, "found") - med(n, 4, "found")) / 12, 1)
        print("found_rec", n, res["found_rec"][n], "ns/record", flush=True)
    for n in (32, 64):   # records of 24 keys: 8 of them add <= 192 entries (n + 192 <= 256)
        res["found_small_rec"][n] = round((med(n, 8, "found24") - med(n, 2, "found24")) / 6, 1)
        print("found_small_rec", n, res["found_small_rec"][n], "ns/record", flush=True)
    for n in (0, 128, 256, 512, 768):
        t = [one_call(n, 4, "insert", rep) for rep in range(args.reps)]
        res["insert"][n] = round(float(np.median([a / b for a, b in t])), 1)
        print("insert", n, res["insert"][n], "ns/Inc", flush=True)
    # Per ROW at full occupancy of the 256-entry kernel (the throughput side of the model):
    # R rows, each with an image of 32 entries, get one record of one existing key; the
    # difference of the launch times for R2 and R1 rows / (R2 - R1) is one row's share of
    # the chip: its setup (descriptor, record references, header, image load, key map,
    # write-back) with 7 waves per SIMD interleaved.
    def rows_call(R, rep):
        rng = np.random.RandomState(77 + rep)
        srv = psa.Server(0, 1, [1, 99])
        srv.CreateTable(3, psa.TableInfo(row_kind=psa.ROW_SORTED_MAP, dtype=psa.I32, row_capacity=K,
                                         oplog_dense_serialized=False, max_rows=R, max_entries=K))
        have = np.arange(32, dtype=np.int32)
        fill = wire.sparse_stream_np(3, 4, [(r, have, np.full(32, 5, np.int32)) for r in range(R)])
        srv.ApplyOpLogUpdateVersion(fill.tobytes(), fill.size, 99, 0)
        one = wire.sparse_stream_np(3, 4, [(int(r), np.array([int(rng.randint(32))], np.int32),
                                            np.ones(1, np.int32)) for r in rng.permutation(R)])
        d = torch.from_numpy(one).cuda()
        torch.cuda.synchronize()
        srv.timing(2)
        srv.timing_reset()
        srv.apply_device([(d.data_ptr(), d.numel(), 1, 0)])
        srv.sync()
        ms, _ = srv.timing_read("ordered_apply")
        srv.close()
        return ms * 1e6
    r1, r2 = 7168 * 2, 7168 * 8
    t1 = float(np.median([rows_call(r1, rep) for rep in range(args.reps)]))
    t2 = float(np.median([rows_call(r2, rep) for rep in range(args.reps)]))
    res["row_share"] = round((t2 - t1) / (r2 - r1), 2)
    print("row_share", res["row_share"], "ns per row at full occupancy", flush=True)
    out = {"what": "ns per record of 64 found keys in one wave's dependent chain (one row, one wave; median of reps; "
                   "difference of two ordered_apply launch times, so the launch's fixed part cancels): found_rec on "
                   "the 1,024-entry register image (16 vs 4 records), found_small_rec on the 256-entry image (8 vs 2 "
                   "records of 24 keys); insert: ns per new key (4 records x 64 new keys, the image growing n -> n + 256, launch "
                   "time / Incs).",
           "found_rec_ns": res["found_rec"], "found_small_rec_ns": res["found_small_rec"], "insert_ns": res["insert"],
           "row_share_ns": res["row_share"],
           "row_share_what": "one row's share of the chip at full occupancy of the 256-entry kernel: launch time "
                             "difference of 57,344 and 14,336 one-record rows (images of 32 entries) per row"}
    print(json.dumps(out))
    if args.out:
        json.dump(out, open(args.out, "w"), indent=1)


if __name__ == "__main__":
    main()
