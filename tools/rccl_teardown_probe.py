"""Diagnostic: what the garbage collector frees after a captured RCCL step (round-4 teardown abort).

tests/test_gpu_ddp.py's world-1 RCCL case aborted inside ddp.teardown's gc.collect() (after the
graph with the captured collectives had gone out of scope).  This probe replays the test's steps
in a process of its own, lists the types of every object the collector would free
(gc.DEBUG_SAVEALL keeps them in gc.garbage), then frees them in stages with a line before each,
so the last line printed before an abort names what the abort came from.
"""

from __future__ import annotations

import collections
import gc
import os
import socket
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "cgr-mpnn-3d_amd"), os.path.join(REPO, "tests")]

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402


def say(*a):
    print("[probe]", *a, flush=True)


def main():
    from test_gpu_ddp import _captured, _grads, _model

    from cgr_mpnn_3D._amd import native
    from cgr_mpnn_3D._amd.ddp import install_grad_allreduce, teardown

    native.load().cgr_debug_abort_backtrace(1)  # an abort names its thread and native stack
    dev = torch.device("cuda:0")
    m, data = _model(dev, D=4, H=400, skip=False)
    ref = _captured(m, data)
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    store = dist.TCPStore("127.0.0.1", port, 1, True)
    dist.init_process_group("nccl", store=store, rank=0, world_size=1, device_id=dev)
    install_grad_allreduce(m)
    eager = _grads(m, data)
    gc.collect()  # cycles from before the captured step
    gc.set_debug(gc.DEBUG_SAVEALL)
    cap = _captured(m, data)
    ok = all(torch.equal(a, r) and torch.equal(c, r) for a, c, r in zip(eager, cap, ref))
    say("bitwise", ok)
    torch.cuda.synchronize()
    n = gc.collect()
    kinds = collections.Counter(type(o).__module__ + "." + type(o).__qualname__ for o in gc.garbage)
    say("collectable objects after the captured step:", n)
    for k, c in kinds.most_common(40):
        say(f"  {c:5d} {k}")
    interesting = [o for o in gc.garbage if "torch" in type(o).__module__ or "cgr" in
                   type(o).__module__ or "Event" in type(o).__name__ or "Graph" in
                   type(o).__name__ or "Stream" in type(o).__name__]
    say("torch / cgr objects among them:", len(interesting))
    for o in interesting[:40]:
        say("  ", type(o), getattr(o, "shape", ""), getattr(o, "device", ""))
    gc.set_debug(0)
    del interesting
    # free in stages: tensors first, then everything else
    tens = [o for o in gc.garbage if isinstance(o, torch.Tensor)]
    say("freeing", len(tens), "tensors")
    for t in tens:
        gc.garbage.remove(t)
    del tens
    gc.collect()
    torch.cuda.synchronize()
    say("tensors freed; freeing the rest:", len(gc.garbage))
    gc.garbage.clear()
    gc.collect()
    torch.cuda.synchronize()
    say("all freed; ddp.teardown (hook closed, process group destroyed, then collected)")
    teardown(m, graphs_released=True)
    say("destroyed")


if __name__ == "__main__":
    main()
