"""GPU: the data-parallel gradient exchange on the HIP path (cgr_mpnn_3D._amd.ddp).

The native backward records one ready event per gradient bucket (include/cgr_mpnn3d.h,
CGR_GRAD_BUCKETS) and GradAllReduce starts each bucket's collective on a communication stream as
soon as its event fires.  What is checked here, on one GPU:
  * a bucket op that doubles the bucket in place: every gradient comes out exactly 2x the
    hook-free gradient, eagerly and inside a captured training step -- each event fired after its
    bucket's last write (an early event would let a later write overwrite the doubled values) and
    the buckets cover every parameter once;
  * a world-1 RCCL process group (backend "nccl"): the real all_reduce(SUM) of every bucket
    inside a captured step leaves the gradients bitwise equal to the run without the hook, and
    ddp.teardown then ends it in bench.py's order (graph dropped, sync, hook closed, destroy, and
    only then a collection) -- with no collection of its own beforehand, after other GPU work has
    left garbage behind.  It runs in a child process with the native abort backtrace installed
    (cgr_debug_abort_backtrace), so an abort names its thread and cannot end the suite;
  * bench.py's distributed path itself (--force-dist 1: RCCL world 1, the collectives captured
    with the step, ddp.teardown after the JSON line), exit status 0;
  * two real ranks (two processes sharing the one GPU, gloo): each runs the native forward /
    backward on its shard of the cfg2 batch with install_grad_allreduce; the all-reduced gradients
    are bitwise identical on both ranks and equal the whole-batch native gradient (1e-4).
Reference: the single-device step of train.py:109-114 / trainer.py:138-144.
"""

import os
import socket
import sys

import pytest
import torch
import torch.distributed as dist

if __name__ == "__main__":  # child process (_rccl_child): the paths conftest.py sets for pytest
    _repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path[:0] = [_repo, os.path.join(_repo, "cgr-mpnn-3d_amd")]

from cgr_mpnn_3D._amd.ddp import install_grad_allreduce, remove_grad_allreduce
from cgr_mpnn_3D._amd.synth import make_batch
from cgr_mpnn_3D.models.GNN import GNN

pytestmark = pytest.mark.gpu


def _model(dev, D=3, H=128, skip=True):
    torch.manual_seed(0)
    b = make_batch(24, n_atoms=30, n_bonds=30, n_mace=32, seed=91)
    m = GNN(b.x.shape[1], 14, depth=D, hidden_sizes=[H] * D, dropout_ps=[0.0] * D,
            use_learnable_skip=skip).to(dev).train()
    return m, b.to_torch(dev)


def _grads(m, data):
    params = list(m.parameters())
    pred = m(data)
    loss = torch.nn.MSELoss(reduction="sum")(pred, data.y)
    return [g.detach().clone() for g in torch.autograd.grad(loss, params)]


def _captured(m, data):
    params = list(m.parameters())

    def step():
        pred = m(data)
        loss = torch.nn.MSELoss(reduction="sum")(pred, data.y)
        return torch.autograd.grad(loss, params)

    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        for _ in range(2):
            step()
    torch.cuda.current_stream().wait_stream(s)
    g = torch.cuda.CUDAGraph()
    # thread-local: a live process group's watchdog thread queries events during the capture
    with torch.cuda.graph(g, capture_error_mode="thread_local"):
        out = step()
    g.replay()
    torch.cuda.synchronize()
    return [t.detach().clone() for t in out]


def test_bucket_events_order_every_bucket_eager_and_captured(cuda_device):
    m, data = _model(cuda_device)
    ref = _grads(m, data)
    install_grad_allreduce(m, op=lambda t: t.mul_(2.0))
    try:
        eager = _grads(m, data)
        torch.cuda.synchronize()
        for a, r in zip(eager, ref):
            assert torch.equal(a, 2.0 * r)
        cap = _captured(m, data)
        for a, r in zip(cap, ref):
            assert torch.equal(a, 2.0 * r)
    finally:
        remove_grad_allreduce(m)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _rccl_world1_child():
    """The world-1 RCCL case in bench.py's order, after other GPU work has left garbage (run as a
    child process: test_world1_rccl_...)."""
    from cgr_mpnn_3D._amd import native
    from cgr_mpnn_3D._amd.ddp import teardown

    native.load().cgr_debug_abort_backtrace(1)
    dev = torch.device("cuda:0")
    torch.cuda.set_device(dev)
    # earlier work, as the tests before this one leave it: a captured step with a bucket op,
    # models, arenas and an exception traceback (a reference cycle holding tensors), none of it
    # collected before the communicator exists
    m0, d0 = _model(dev)
    install_grad_allreduce(m0, op=lambda t: t.mul_(2.0))
    _captured(m0, d0)
    remove_grad_allreduce(m0)
    try:
        keep = _grads(m0, d0)  # noqa: F841
        raise ValueError("cycle")
    except ValueError as e:
        junk = [e]  # noqa: F841  (frame <-> traceback cycle over keep, m0, d0)
    del m0, d0, keep, junk

    m, data = _model(dev, D=4, H=400, skip=False)
    ref = _captured(m, data)
    store = dist.TCPStore("127.0.0.1", _free_port(), 1, True)
    dist.init_process_group("nccl", store=store, rank=0, world_size=1, device_id=dev)
    install_grad_allreduce(m)
    eager = _grads(m, data)
    cap = _captured(m, data)  # its graph (with the captured collectives) is gone on return
    ok = all(torch.equal(a, r) and torch.equal(c, r) for a, c, r in zip(eager, cap, ref))
    assert m._grad_bucket_hook.captured > 0  # the hook knows it recorded collectives
    teardown(m, graphs_released=True)
    assert not dist.is_initialized() and m._grad_bucket_hook is None
    print(f"RCCL_WORLD1_BITWISE={ok}", flush=True)


def _run_child(args, timeout=240, env=None):
    import subprocess

    p = subprocess.run([sys.executable, "-u"] + args, capture_output=True, text=True,
                       timeout=timeout, env=dict(os.environ, **(env or {})))
    return p.returncode, p.stdout + p.stderr


def test_world1_rccl_allreduce_inside_captured_step_is_bitwise_identity(cuda_device):
    rc, out = _run_child([os.path.abspath(__file__), "--rccl-world1"])
    assert rc == 0, out[-4000:]
    assert "RCCL_WORLD1_BITWISE=True" in out, out[-4000:]


def test_bench_distributed_path_rccl_world1_exits_clean(cuda_device):
    import json

    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    rc, out = _run_child(
        [os.path.join(repo, "bench.py"), "--force-dist", "1", "--config", "cfg1", "--steps", "5",
         "--warmup", "3", "--profile-steps", "0", "--collate-bench", "0", "--infer-bench", "0",
         "--cpu-baseline", "0"],
        env={"MASTER_ADDR": "127.0.0.1", "MASTER_PORT": str(_free_port())})
    assert rc == 0, out[-4000:]
    line = [ln for ln in out.splitlines() if ln.startswith("{")][-1]
    j = json.loads(line)
    assert j["value"] > 0 and j["config"]["parallelism"] == "dp1", j


def _two_rank_child(out_dir):
    """One rank of the two-process run (RANK / WORLD_SIZE / MASTER_* from the parent)."""
    import numpy as np

    from cgr_mpnn_3D._amd.ddp import shard_batch, teardown
    from cgr_mpnn_3D._amd.synth import CONFIGS

    from cgr_mpnn_3D._amd import native

    native.load().cgr_debug_abort_backtrace(1)
    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    dev = torch.device("cuda:0")
    torch.cuda.set_device(dev)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    c = CONFIGS["cfg2"]
    b = make_batch(c["num_graphs"], c["n_atoms"], c["n_bonds"], c["n_mace"], seed=1234)
    D, H = c["depth"], c["hidden"]
    torch.manual_seed(0)
    m = GNN(b.x.shape[1], 14, depth=D, hidden_sizes=[H] * D, dropout_ps=[0.0] * D).to(dev).train()
    names = [k for k, _ in m.named_parameters()]
    if rank == 0:  # the whole batch on one process, no hook: what the sum must equal
        whole = _grads(m, b.to_torch(dev))
        np.savez(os.path.join(out_dir, "whole.npz"),
                 **{k: g.cpu().numpy() for k, g in zip(names, whole)})
    install_grad_allreduce(m)
    reduced = _grads(m, shard_batch(b, rank, world).to_torch(dev))
    torch.cuda.synchronize()
    np.savez(os.path.join(out_dir, f"rank{rank}.npz"),
             **{k: g.cpu().numpy() for k, g in zip(names, reduced)})
    teardown(m)
    print(f"RANK{rank}_OK", flush=True)


def test_two_ranks_on_one_gpu_allreduce_equals_whole_batch(cuda_device, tmp_path):
    import subprocess

    import numpy as np

    port = _free_port()
    procs = []
    for r in range(2):
        env = dict(os.environ, MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(r),
                   WORLD_SIZE="2", LOCAL_RANK=str(r))
        procs.append(subprocess.Popen(
            [sys.executable, "-u", os.path.abspath(__file__), "--two-rank", str(tmp_path)],
            env=env, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True))
    outs = []
    try:
        for p in procs:
            outs.append(p.communicate(timeout=240)[0])
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
    for r, (p, o) in enumerate(zip(procs, outs)):
        assert p.returncode == 0 and f"RANK{r}_OK" in o, o[-3000:]
    whole = np.load(tmp_path / "whole.npz")
    g0, g1 = np.load(tmp_path / "rank0.npz"), np.load(tmp_path / "rank1.npz")
    for k in whole.files:
        assert np.array_equal(g0[k], g1[k]), k  # every rank holds the same summed gradient
        ref = whole[k].astype(np.float64)
        err = np.abs(g0[k] - ref).max() / (np.abs(ref).max() + 1e-30)
        assert err <= 1e-4, (k, err)


if __name__ == "__main__" and "--two-rank" in sys.argv:
    _two_rank_child(sys.argv[sys.argv.index("--two-rank") + 1])
if __name__ == "__main__" and "--rccl-world1" in sys.argv:
    _rccl_world1_child()
