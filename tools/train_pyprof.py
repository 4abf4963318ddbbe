"""Where the host time of one eager training step goes (train.py's default model and batch:
depth 3, hidden 300, 32 reactions; fwd + MSELoss(sum) + bwd + FusedAdam): the step's host
enqueue time, a cProfile of the main thread, a second cProfile of GNNFunction.backward (it runs
on the autograd engine's device thread, which the first does not see), and the host time of each
native enqueue call alone."""

import cProfile
import ctypes
import os
import pstats
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "cgr-mpnn-3d_amd"))
sys.path.insert(0, REPO)

import torch  # noqa: E402


def main():
    from cgr_mpnn_3D._amd import functional as F
    from cgr_mpnn_3D._amd import native
    from cgr_mpnn_3D._amd.loss import MSELoss
    from cgr_mpnn_3D._amd.optim import FusedAdam
    from cgr_mpnn_3D._amd.synth import CONFIGS, make_batch
    from cgr_mpnn_3D.models.GNN import GNN

    cfg = next((a for a in sys.argv[1:] if not a.startswith("--")), "train_default")
    c = CONFIGS[cfg]
    dev = torch.device("cuda:0")
    b = make_batch(c["num_graphs"], c["n_atoms"], c["n_bonds"], c["n_mace"], seed=1234)
    data = b.to_torch(dev)
    D, H = c["depth"], c["hidden"]
    torch.manual_seed(0)
    m = GNN(b.x.shape[1], 14, depth=D, hidden_sizes=[H] * D, dropout_ps=[0.02] * D,
            use_learnable_skip=c["learnable_skip"]).to(dev).train()
    opt = FusedAdam(m.parameters(), lr=1e-3, amsgrad=True)
    loss_fn = MSELoss(reduction="sum")

    def step():
        opt.zero_grad(set_to_none=True)
        loss = loss_fn(m(data), data.y)
        loss.backward()
        opt.step()

    def host_us(fn, n=300):
        for _ in range(20):
            fn()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for i in range(n):
            fn()
            if i % 25 == 24:
                torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        torch.cuda.synchronize()
        return round(dt / n * 1e6, 1)

    if "--steps-only" in sys.argv:  # for rocprofv3 --runtime-trace: 500 eager steps, nothing else
        for i in range(500):
            step()
            if i % 25 == 24:
                torch.cuda.synchronize()
        torch.cuda.synchronize()
        return
    print(f"{cfg}: step wall (sync every 25) {host_us(step)} us")
    t0 = time.perf_counter()
    for _ in range(200):
        step()
    h = (time.perf_counter() - t0) / 200
    torch.cuda.synchronize()
    print(f"  host enqueue {h * 1e6:.1f} us per step")

    # pieces alone
    def fwd_only():
        with torch.no_grad():
            pass
    y = m(data)
    loss = loss_fn(y, data.y)
    print("  forward (GNN.forward + apply)      ", host_us(lambda: m(data)), "us")
    print("  loss forward                       ", host_us(lambda: loss_fn(y, data.y)), "us")
    print("  zero_grad                          ", host_us(lambda: opt.zero_grad(True)), "us")

    def fb():
        m(data).sum().backward()
    print("  forward+sum+backward               ", host_us(fb), "us")
    fb()
    print("  opt.step                           ", host_us(opt.step), "us")
    print("  opt.step (unwrapped)               ", host_us(lambda: FusedAdam.step.__wrapped__(opt)
                                                         if hasattr(FusedAdam.step, "__wrapped__")
                                                         else opt.step()), "us")
    # the native calls alone, through the same ctypes arguments
    lib = native.load()
    orig_fwd, orig_bwd = lib.cgr_gnn_forward, lib.cgr_gnn_backward
    acc = {"fwd": [], "bwd": []}

    class Timed:
        def __init__(self, fn, k):
            self.fn, self.k = fn, k

        def __call__(self, *a):
            t = time.perf_counter()
            r = self.fn(*a)
            acc[self.k].append(time.perf_counter() - t)
            return r
    # F's lib is native.load()'s object: patch its attributes
    lib.cgr_gnn_forward = Timed(orig_fwd, "fwd")
    lib.cgr_gnn_backward = Timed(orig_bwd, "bwd")
    orig_backward = F.GNNFunction.backward
    bacc = []
    pr_b = cProfile.Profile()

    def timed_backward(ctx, dy):
        t = time.perf_counter()
        pr_b.enable()
        r = orig_backward(ctx, dy)
        pr_b.disable()
        bacc.append(time.perf_counter() - t)
        return r
    F.GNNFunction.backward = staticmethod(timed_backward)
    for i in range(300):
        step()
        if i % 25 == 24:
            torch.cuda.synchronize()
    torch.cuda.synchronize()
    import statistics as s
    print("  native cgr_gnn_forward call        ", round(s.median(acc["fwd"]) * 1e6, 1), "us")
    print("  native cgr_gnn_backward call       ", round(s.median(acc["bwd"]) * 1e6, 1), "us")
    print("  GNNFunction.backward (engine thr.) ", round(s.median(bacc) * 1e6, 1), "us")
    lib.cgr_gnn_forward, lib.cgr_gnn_backward = orig_fwd, orig_bwd
    F.GNNFunction.backward = staticmethod(orig_backward)
    print("=== backward thread profile")
    pstats.Stats(pr_b).sort_stats("tottime").print_stats(20)
    pr = cProfile.Profile()
    pr.enable()
    for i in range(1000):
        step()
        if i % 20 == 19:
            torch.cuda.synchronize()
    pr.disable()
    torch.cuda.synchronize()
    print("=== main thread profile")
    pstats.Stats(pr).sort_stats("tottime").print_stats(30)


if __name__ == "__main__":
    main()
