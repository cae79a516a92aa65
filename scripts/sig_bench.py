#!/usr/bin/env python3
"""Throughput of the batched secp256k1 kernels (libbftsig) on one GPU: sign and recover of a batch
resident in HBM, timed with HIP events on the launch stream. Prints one JSON line."""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "consensus-rs_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=262_144)
    ap.add_argument("--reps", type=int, default=3)
    args = ap.parse_args()
    import torch
    from bftsim.sig import Signer
    sg = Signer(0)
    g = torch.Generator().manual_seed(1)
    keys = 64
    secs = torch.randint(0, 256, (keys, 32), dtype=torch.uint8, generator=g)
    secs[:, 0] &= 0x7f
    digs = torch.randint(0, 256, (args.n, 32), dtype=torch.uint8, generator=g).cuda()
    kidx = (torch.arange(args.n, dtype=torch.int32) % keys).cuda()
    secs = secs.cuda()
    out = {}
    sig, ok = sg.sign(secs, digs, key_index=kidx)      # warm-up
    sg.recover(digs, sig, want_pub=False)
    torch.cuda.synchronize()
    for name, fn in (("sign", lambda: sg.sign(secs, digs, key_index=kidx)),
                     ("recover", lambda: sg.recover(digs, sig, want_pub=False))):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(args.reps):
            fn()
        e1.record()
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / args.reps
        out[name] = {"ms": ms, "per_s": args.n / (ms / 1e3)}
    print(json.dumps({"n": args.n, **out}))


if __name__ == "__main__":
    main()
