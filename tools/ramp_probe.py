"""Diagnostic (round 6): does a kernel run slower for its first launches after the
device idled?  After `--idle-s` of host sleep, times each of `--n` back-to-back launches (one HIP
event pair per launch on the launch stream) of
  * an HBM-bound copy (256 MB -> 256 MB, beyond the 256 MB Infinity Cache once both count), and
  * an MFMA-bound bf16 GEMM (4096^3),
so a ramp of the memory side can be told from one of the compute side.  Prints one JSON line.
"""

import json
import time

import torch


def timed(fn, n):
    s = torch.cuda.current_stream()
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(n + 1)]
    for i in range(n):
        ev[i].record(s)
        fn()
    ev[n].record(s)
    torch.cuda.synchronize()
    return [round(ev[i].elapsed_time(ev[i + 1]) * 1e3, 1) for i in range(n)]


def main():
    import argparse

    ap = argparse.ArgumentParser()
    ap.add_argument("--idle-s", type=float, default=1.0)
    ap.add_argument("--n", type=int, default=80)
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    src = torch.randn(64 * 2**20, device=dev)  # 256 MB
    dst = torch.empty_like(src)
    A = torch.randn(4096, 4096, device=dev, dtype=torch.bfloat16)
    B = torch.randn(4096, 4096, device=dev, dtype=torch.bfloat16)
    C = torch.empty(4096, 4096, device=dev, dtype=torch.bfloat16)
    dst.copy_(src)
    torch.matmul(A, B, out=C)
    torch.cuda.synchronize()
    out = {}
    for name, fn in (("copy_256MB", lambda: dst.copy_(src)),
                     ("gemm_bf16_4096", lambda: torch.matmul(A, B, out=C)),
                     ("copy_256MB_again", lambda: dst.copy_(src))):
        time.sleep(a.idle_s)
        us = timed(fn, a.n)
        out[name] = {"first5_us": us[:5], "launch_10_19_mean": round(sum(us[10:20]) / 10, 1),
                     "last20_mean": round(sum(us[-20:]) / 20, 1), "all_us": us}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
