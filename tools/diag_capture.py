"""Bisect HIP-graph capture of the native path: stages run in order, each prints before/after."""

import ctypes
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "cgr-mpnn-3d_amd"))
sys.path.insert(0, REPO)

if os.environ.get("IMPORT_SCIPY"):
    import scipy.sparse  # noqa: F401
    import scipy.special  # noqa: F401
import torch  # noqa: E402

from cgr_mpnn_3D._amd import native  # noqa: E402
from cgr_mpnn_3D._amd.functional import _batch_struct, make_config  # noqa: E402
from cgr_mpnn_3D._amd.synth import make_batch  # noqa: E402
from cgr_mpnn_3D.models.GNN import GNN  # noqa: E402


def say(*a):
    print("[diag]", *a, flush=True)


def capture(fn, name):
    say("begin", name)
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        fn()
    torch.cuda.current_stream().wait_stream(s)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        fn()
    say("captured", name)
    g.replay()
    torch.cuda.synchronize()
    say("ok", name)
    return g


def main():
    stages = sys.argv[1].split(",") if len(sys.argv) > 1 else ["seg", "prep", "fwd", "fwdgrad",
                                                                "fwdbwd"]
    dev = torch.device("cuda:0")
    lib = native.load()
    B = int(os.environ.get("B", "8"))
    H = int(os.environ.get("H", "64"))
    D = int(os.environ.get("D", "2"))
    b = make_batch(B, seed=1)
    data = b.to_torch(dev)
    torch.manual_seed(0)
    m = GNN(b.x.shape[1], 14, depth=D, hidden_sizes=[H] * D, dropout_ps=[0.0] * D).to(dev)
    N, E = b.x.shape[0], b.edge_index.shape[1]
    cfg = make_config(b.x.shape[1], 14, H, D, 0, False)
    arena = torch.empty(lib.cgr_gnn_arena_bytes(ctypes.byref(cfg), N, E, B), dtype=torch.uint8,
                        device=dev)
    bs = _batch_struct(data.x, data.edge_index, data.edge_attr, data.batch, data.ptr, B)

    vals = torch.randn(1000, 64, device=dev)
    ptr = torch.arange(0, 1001, 10, dtype=torch.int32, device=dev)
    out = torch.empty(100, 64, device=dev)

    def seg():
        native.check(lib.cgr_segment_sum(native.ptr(vals), 64, None, native.ptr(ptr), 100, 64,
                                         native.ptr(out), 64,
                                         native.stream_ptr(dev)))

    def prep():
        native.check(lib.cgr_graph_prep(ctypes.byref(cfg), ctypes.byref(bs), native.ptr(arena),
                                        native.stream_ptr(dev)))

    def fwd():
        with torch.no_grad():
            m(data)

    def fwdgrad():
        m(data).sum()

    def fwdbwd():
        loss = m(data).sum()
        torch.autograd.grad(loss, list(m.parameters()))

    def testbody():
        params = list(m.parameters())

        def step():
            pred = m(data)
            loss = torch.nn.MSELoss(reduction="sum")(pred, data.y)
            gs = torch.autograd.grad(loss, params)
            return pred, gs

        say("testbody eager")
        step()
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            for _ in range(2):
                step()
        torch.cuda.current_stream().wait_stream(s)
        g = torch.cuda.CUDAGraph()
        say("testbody capture")
        with torch.cuda.graph(g):
            step()
        say("testbody replay")
        g.replay()
        torch.cuda.synchronize()

    table = dict(seg=seg, prep=prep, fwd=fwd, fwdgrad=fwdgrad, fwdbwd=fwdbwd)
    if "testbody" in stages:
        testbody()
        say("testbody ok")
        return
    for st in stages:
        capture(table[st], st)
    say("all ok")


if __name__ == "__main__":
    main()
