"""Diagnostic: what the shader clock did while bench.py's timed steps ran.

Replays bench.py's sequence for one configuration -- max(3, W) eager steps, 3 side-stream steps,
capture, W replays, then the timed K steps, then `--blocks` more blocks of K steps -- with a stamp
kernel (tools/clock_probe.hip) on the step stream before every replay.  Each stamp records the
real-time clock (100 MHz) and reads the shader clock over a short spin (d s_memtime /
d s_memrealtime x 100 MHz, MI355X_MICROARCH.md 'DVFS give-back' item 6), so the record gives
every step's device duration and the clock the chip held around it.  (A sampler on a stream of
its own would share a hardware queue with the step and serialise it.)

    python tools/clock_gap.py [--steps 20 --warmup 5 --blocks 10 --config cfg2]
"""

import argparse
import ctypes
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "cgr-mpnn-3d_amd"))
sys.path.insert(0, REPO)

import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--blocks", type=int, default=10)
    ap.add_argument("--config", default="cfg2")
    ap.add_argument("--spin-ticks", type=int, default=200, help="2 us at 100 MHz")
    ap.add_argument("--pre-spin-ms", type=float, default=0.0,
                    help="replay steps for this long (untimed) before the timed block")
    args = ap.parse_args()

    from cgr_mpnn_3D._amd.loss import MSELoss
    from cgr_mpnn_3D._amd.optim import FusedAdam
    from cgr_mpnn_3D._amd.synth import CONFIGS, make_batch
    from cgr_mpnn_3D.models.GNN import GNN

    probe = ctypes.CDLL(os.path.join(REPO, "tools", "_build", "libclockprobe.so"))
    dev = torch.device("cuda:0")
    torch.cuda.set_device(dev)
    c = CONFIGS[args.config]
    D, H = c["depth"], c["hidden"]
    b = make_batch(c["num_graphs"], c["n_atoms"], c["n_bonds"], c["n_mace"], seed=1234)
    data = b.to_torch(dev)
    B = b.num_graphs
    torch.manual_seed(0)
    model = GNN(b.x.shape[1], 14, depth=D, hidden_sizes=[H] * D, dropout_ps=[0.02] * D,
                use_learnable_skip=c["learnable_skip"]).to(dev).train()
    opt = FusedAdam(model.parameters(), lr=1e-3, amsgrad=True)
    loss_fn = MSELoss(reduction="sum")

    def step():
        opt.zero_grad(set_to_none=True)
        loss = loss_fn(model(data), data.y)
        loss.backward()
        opt.step()

    main_s = torch.cuda.current_stream(dev)
    nmax = 64 + args.warmup + (args.blocks + 1) * (args.steps + 1) + 4000
    stamps = torch.zeros(4 * nmax, dtype=torch.int64, device=dev)
    names = []

    def stamp(name):
        assert len(names) < nmax
        probe.clock_probe_stamp(ctypes.c_void_p(stamps.data_ptr() + 32 * len(names)),
                                ctypes.c_ulonglong(args.spin_ticks),
                                ctypes.c_void_p(main_s.cuda_stream))
        names.append(name)

    for i in range(max(3, args.warmup)):
        stamp(f"eager{i}")
        step()
    torch.cuda.synchronize()
    s = torch.cuda.Stream()
    s.wait_stream(main_s)
    with torch.cuda.stream(s):
        for _ in range(3):
            step()
    main_s.wait_stream(s)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        step()
    hrep = {}

    def replay(name):
        t = time.perf_counter()
        g.replay()
        hrep[name] = round((time.perf_counter() - t) * 1e6, 1)

    for i in range(args.warmup):
        stamp(f"warm{i}")
        replay(f"warm{i}")
    torch.cuda.synchronize()
    if args.pre_spin_ms > 0:
        t0 = time.perf_counter()
        i = 0
        while time.perf_counter() - t0 < args.pre_spin_ms * 1e-3:
            stamp(f"spin{i}")
            replay(f"spin{i}")
            i += 1
            if i % 20 == 0:
                main_s.synchronize()
        torch.cuda.synchronize()
    host = []
    for blk in range(args.blocks + 1):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for i in range(args.steps):
            stamp(f"b{blk}s{i}")
            replay(f"b{blk}s{i}")
        stamp(f"b{blk}end")
        torch.cuda.synchronize()
        host.append((time.perf_counter() - t0) / args.steps * 1e3)
    torch.cuda.synchronize()
    st = stamps.view(-1, 4)[:len(names)].cpu().tolist()

    def clk(x):
        return (x[3] - x[1]) / (x[2] - x[0]) * 0.1 if x[2] > x[0] else None

    steps = []
    for i in range(len(names) - 1):
        steps.append({"name": names[i], "t_ms": round((st[i][0] - st[0][0]) * 1e-5, 4),
                      "dev_ms": round((st[i + 1][0] - st[i][2]) * 1e-5, 4),
                      "clock_ghz": round(clk(st[i]), 3),
                      "host_replay_us": hrep.get(names[i])})
    out = {"config": args.config, "steps": args.steps, "warmup": args.warmup,
           "pre_spin_ms": args.pre_spin_ms, "blocks": []}
    for blk in range(args.blocks + 1):
        ss = [x for x in steps if x["name"].startswith(f"b{blk}s")]
        out["blocks"].append({"block": "timed" if blk == 0 else blk,
                              "host_ms_per_step": round(host[blk], 4),
                              "dev_ms_per_step": round(sum(x["dev_ms"] for x in ss) / len(ss), 4),
                              "clock_ghz_mean": round(sum(x["clock_ghz"] for x in ss) / len(ss), 3),
                              "clock_ghz_first": ss[0]["clock_ghz"],
                              "dev_ms_first": ss[0]["dev_ms"]})
    out["steps_record"] = steps
    print(json.dumps(out))


if __name__ == "__main__":
    main()
