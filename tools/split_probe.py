"""C4's chunked pipeline on one GPU with the split kept (split_single): the device split of
each 2 GiB chunk, the rank's own sub-stream applied from the send slot, parity against the
seeds.  Prints the exchange_measure JSON (split_host_ms_per_step: the split's wall time).
usage: python tools/split_probe.py [--rows 10000000] [--steps 3]"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=10_000_000)
    ap.add_argument("--steps", type=int, default=3)
    args = ap.parse_args()
    import torch
    import bench
    torch.cuda.set_device(0)
    m = bench.exchange_measure(args.rows, 1024, args.steps, 1, 1, 0, 0, split_single=True)
    print(json.dumps({k: m[k] for k in ("ms_per_step", "parity", "split_host_ms_per_step", "exchange_wait_ms_per_step",
                                        "apply_wait_ms_per_step", "apply_kernel_ms_per_chunk", "chunks_per_step")}),
          flush=True)


if __name__ == "__main__":
    main()
