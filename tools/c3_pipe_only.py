"""One pipelined C3 measurement alone (bench.c3_measure with pipeline=True), for a rocprofv3
kernel trace whose steady state is easy to cut out: the timed pass, then its two event
passes.  Usage: python tools/c3_pipe_only.py [--indexed] [--steps K] [--warmup W]"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: F401  (HIP runtime first, as bench.py does)
import bench

sys.argv = [sys.argv[0]] + sys.argv[1:]
args = bench.parse()
m = bench.c3_measure(args, args.indexed, args.steps, args.warmup, 0.0, pipeline=True)
print(json.dumps({k: m[k] for k in ("value", "ms_per_step", "ordered_apply_ms_per_step", "host_enqueue_ms_per_step")}))
