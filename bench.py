"""Benchmark: reactions/s of the CGR-MPNN-3D training step on 1..8 MI355X (one process per GPU).

    python bench.py [--gpus N --steps K --warmup W]                      (N = 1)
    python -m torch.distributed.run --nnodes=1 --nproc-per-node N --master-addr 127.0.0.1 \
        --master-port P bench.py --gpus N --steps K --warmup W          (N > 1, RCCL)

A step is one pass of the hot path over one synthetic, HBM-resident batch of BASELINE config 2
(256 reactions per GPU, 30 atoms / 60 directed edges each, F = 846, Fe = 14, depth 4, hidden
400): forward, MSELoss(sum), backward (native), RCCL all-reduce(SUM) of the flat gradient
bucket when N > 1, Adam(amsgrad) step (train.py:117-121; the fused native FusedAdam by default,
--optimizer torch for torch.optim.Adam).  Per-GPU work is fixed (weak scaling).
Rank 0 prints ONE JSON line.  See DESIGN.md "Measurement".
"""

from __future__ import annotations

import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(REPO, "cgr-mpnn-3d_amd"))
sys.path.insert(0, REPO)

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

METRIC = "reactions/sec (fwd+bwd) depth=4 hidden=400 T1x batch; 1/2/4/8 MI355X"
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec
FP32_MFMA_PEAK_TFLOPS = 157.3  # MI355X_MICROARCH.md: v_mfma_f32_*_f32 dense peak
BF16_MFMA_PEAK_TFLOPS = 2516.8  # 16 x the fp32 MFMA rate (MI355X_MICROARCH.md, dense)


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=30)
    ap.add_argument("--config", default="cfg2",
                    choices=["cfg1", "cfg2", "cfg4", "cfg5", "train_default", "sweep_b16",
                             "sweep_b64", "sweep_d5", "sweep_max"])
    ap.add_argument("--graph", type=int, default=-1,
                    help="capture the step in a HIP graph (1/0; -1 = auto: on for N = 1)")
    ap.add_argument("--loss", default="fused", choices=["fused", "torch"],
                    help="MSELoss(sum): native cgr_mse_loss (default) or torch.nn.MSELoss")
    ap.add_argument("--optimizer", default="fused", choices=["fused", "torch"],
                    help="fused: cgr FusedAdam (one native launch); torch: torch.optim.Adam")
    ap.add_argument("--dropout", type=float, default=0.02,
                    help="dropout p per layer (train.py default 0.02)")
    ap.add_argument("--dist-backend", default="nccl", choices=["nccl", "gloo"],
                    help="nccl (= RCCL) for the real run; gloo only to rehearse the N>1 code path "
                         "with several ranks on one GPU")
    ap.add_argument("--force-dist", type=int, default=0,
                    help="initialise the process group and the gradient all-reduce even at N=1 "
                         "(rehearses the collective inside a captured graph on one GPU)")
    ap.add_argument("--collate-bench", type=int, default=1,
                    help="also measure on-device collation (SURVEY §8(f) rank 1), N=1 only")
    ap.add_argument("--infer-bench", type=int, default=1,
                    help="also measure the eval forward (SURVEY §8(f) rank 3), N=1 only")
    ap.add_argument("--cpu-baseline", type=int, default=1)
    ap.add_argument("--cpu-seconds", type=float, default=10.0,
                    help="per thread setting (the baseline runs at two)")
    ap.add_argument("--profile-steps", type=int, default=10,
                    help="instrumented steps (HIP events per kernel class) after the timed run")
    ap.add_argument("--min-warmup-ms", type=float, default=200.0,
                    help="after the W warmup steps, keep running untimed steps until the device "
                         "has spent this long in back-to-back steps (steady state; 0 = off)")
    ap.add_argument("--diag-blocks", type=int, default=0,
                    help="diagnostic: time this many further blocks of --steps steps after the "
                         "timed one (per-step HIP events); not part of `value`")
    ap.add_argument("--traffic-json", default=os.path.join(REPO, "profiles", "traffic.json"))
    return ap.parse_args()


# ------------------------------------------------------------------------------------------------
# algorithmic work per LAUNCH of each kernel class (DESIGN.md "Roofline accounting").  Bytes count
# each operand once (gathered rows of an N-row table count as the table), fp32 = 4 B, int32 index
# = 4 B; flops = 2 per multiply-add.  Classes match the native ProfScope names; every launch of a
# class has the same shape, so (per-launch work) / (average launch time) is the achieved rate.
# ------------------------------------------------------------------------------------------------
def algorithmic_work(N, E, B, F, Fe, H, D, relu=True):
    f4, i4 = 4.0, 4.0
    pre = 0 if relu else 1       # ReLU's derivative is read off the output; others keep pre-act
    w = {}

    def add(name, launches, flops, nbytes):
        w[name] = dict(launches=launches, flops=float(flops), bytes=float(nbytes))

    # forward
    add("gemm_nt_x", 1, 2.0 * N * F * 2 * H, f4 * (N * F + 2 * H * F + 2 * N * H))
    add("edge_init_fwd", 1, 2.0 * E * Fe * H,
        f4 * (N * H + E * Fe + Fe * H + H + E * H * (1 + pre)) + i4 * E)
    # edge init fused with a_0 = segsum_dst(h0) (H <= 512)
    add("edge_init_seg_fwd", 1, 2.0 * E * Fe * H + E * H,
        f4 * (N * H + E * Fe + Fe * H + H + E * H * (1 + pre) + N * H) + i4 * (E + N + 1))
    seg_dst = f4 * (E * H + N * H) + i4 * (N + 1)
    add("segsum_dst_fwd", D + 1, E * H, seg_dst)
    add("gemm_nt_layer_fwd", D, 2.0 * E * H * H,
        f4 * (N * H + E * H + E * H + H * H + H + E * H * (1 + pre)) + 2 * i4 * E)
    # the same GEMM with a_{l+1} = segsum_dst(h_{l+1}) summed in its epilogue (EpLayerSeg)
    add("gemm_nt_layer_seg_fwd", D, 2.0 * E * H * H + E * H,
        f4 * (N * H + E * H + E * H + H * H + H + E * H * (1 + pre) + N * H) + 3 * i4 * E)
    add("gemm_nt_readout_fwd", 1, 2.0 * N * H * H, f4 * (N * H + N * H + H * H + H + 2 * N * H))
    add("pool_head_fwd", 1, 2.0 * N * H, f4 * (N * H + B * H + H + B) + i4 * (B + 1))
    # backward
    add("head_bwd", 1, 2.0 * B * H, f4 * (B + B * H + 2 * H))  # dwf = dy^T g, dbf
    # dzn = dy[graph] wf * act'(zn): hn (ReLU mask) read, dzn's e-image written (2 bf16 pieces,
    # the readout TN's operand; fp32 dzn itself is not stored)
    add("readout_act_bwd", 1, 0.0, f4 * (B + H + 2 * N * H) + i4 * N)
    add("gemm_tn_wgrad_readout", 1, 2.0 * N * H * (F + H),
        f4 * (N * H + N * F + N * H + H * (F + H) + H))
    add("gemm_nt_readout_bwd", 1, 2.0 * N * H * H, f4 * (N * H + H * H + N * H))
    # top layer: dh = ds[dst]; dpre written in fp32 and as the layer TN's e-image (2 bf16 pieces)
    add("layer_act_bwd", 1, 0.0, f4 * (N * H + 3 * E * H) + i4 * E)
    add("gemm_tn_wgrad_layer", D, 2.0 * E * H * H,
        f4 * (E * H + N * H + E * H + H * H + H) + 2 * i4 * E)
    # dm = dpre_l W_l with da = segsum_src(dm) and the layer below's activation backward in its
    # epilogue (D - 1 launches: dpre_l rows, W_l, the h mask, dpre_{l-1} written) or the edge-init
    # backward (1: + the D layers' dpre summed into dh0): per launch on average 4 E*H + H*H floats
    add("gemm_nt_layer_bwd_seg", D, 2.0 * E * H * H + E * H,
        f4 * (4 * E * H + H * H) + i4 * (2 * E))
    add("segsum_src_bwd", 1, E * H, seg_dst + i4 * E)  # Gs = segsum_src(dpre0) for dW0[:, :F]
    add("gemm_tn_wgrad_edge", 1, 2.0 * E * H * Fe, f4 * (E * H + E * Fe + H * Fe + H))
    add("gemm_tn_wgrad_node", 1, 2.0 * N * H * F, f4 * (N * H + N * F + H * F))
    # e-images of the weight gradients' shared operand dpre_l for the layers below the top: fp32
    # in, 2 bf16 out (dzn's and the top layer's dpre's are written by their producers, Gs's by
    # segsum_src_bwd)
    add("eimage", max(D - 1, 1), 0.0, f4 * E * H * 2)
    # split-bf16 weight images, once per step: fp32 weights in, three bf16 pieces out
    nw = 2 * H * F + (2 + 2 * D) * H * H
    add("weight_pack", 1, 0.0, (f4 + 3 * 2.0) * nw)
    return w


def mfma_bound(name):
    return name.startswith("gemm")


# bf16 MFMA products per fp32 multiply-add in the shipped build's GEMMs (csrc/gemm_b3.hpp): NT
# GEMMs split both operands into three bf16 pieces (six products), the layer / node / readout
# weight gradients into two (three products); the edge-feature weight gradient (K = Fe = 14)
# stays on the fp32 MFMA (v_mfma_f32_16x16x4_f32)
BF16_PRODUCTS = {"gemm_nt_x": 6, "gemm_nt_layer_fwd": 6, "gemm_nt_layer_seg_fwd": 6,
                 "gemm_nt_readout_fwd": 6, "gemm_nt_layer_bwd_seg": 6, "gemm_nt_readout_bwd": 6,
                 "gemm_tn_wgrad_layer": 3, "gemm_tn_wgrad_node": 3, "gemm_tn_wgrad_readout": 3}


def roofline_entry(name, work, launches, ms_total, traffic):
    """Per-launch roofline of one kernel class: algorithmic work of one launch / its average
    launch duration, against the ceiling the kernel actually runs on.
      * split-bf16 GEMMs: the bf16 matrix-core work they issue (products x algorithmic FLOPs)
        against the dense bf16 MFMA peak -- their fp32-equivalent rate against the fp32 MFMA peak
        can exceed 1 (the fp32 MFMA is not what limits them), so it is reported only as
        `fp32_equivalent`, never as `frac`;
      * fp32-MFMA GEMMs: algorithmic FLOP/s against the fp32 MFMA peak;
      * everything else: algorithmic bytes against HBM.
    Every class also carries `hbm_frac` = algorithmic bytes / time / 8 TB/s beside it."""
    t = ms_total * 1e-3 / launches
    k = BF16_PRODUCTS.get(name)  # None for the "[f32]" / "[tnr]" fallback families
    hbm = work["bytes"] / t / 1e9
    if k:
        ach, peak, unit, bound = k * work["flops"] / t / 1e12, BF16_MFMA_PEAK_TFLOPS, "TFLOP/s", "mfma"
    elif mfma_bound(name):
        ach, peak, unit, bound = work["flops"] / t / 1e12, FP32_MFMA_PEAK_TFLOPS, "TFLOP/s", "mfma"
    else:
        ach, peak, unit, bound = hbm, HBM_PEAK_GBS, "GB/s", "hbm"
    frac = ach / peak
    if frac > 1.0:
        raise RuntimeError(f"roofline framing error: {name} at {frac:.3f} of its peak")
    out = {"kernel": name, "bound": bound, "achieved": round(ach, 3), "peak": peak, "unit": unit,
           "frac": round(frac, 4), "traffic": traffic,
           "hbm_frac": round(hbm / HBM_PEAK_GBS, 4),
           "algorithmic_bytes_per_launch": work["bytes"],
           "algorithmic_flops_per_launch": work["flops"],
           "avg_launch_us": round(t * 1e6, 3), "launches_measured": launches,
           "timing": "HIP events on the launch stream, instrumented serial pass"}
    if k:
        out["bf16_products_per_fp32_fma"] = k
        f32 = work["flops"] / t / 1e12
        out["fp32_equivalent"] = {"achieved": round(f32, 3), "unit": "TFLOP/s",
                                  "vs_fp32_mfma_peak": round(f32 / FP32_MFMA_PEAK_TFLOPS, 4)}
    if traffic:
        out["traffic_over_algorithmic"] = round(traffic / work["bytes"], 3)
    return out


def scatter_add_roofline(edge_index, N, H, dev, reps=50, cold_copies=24, which=None):
    """The path's scatter-add (PyG propagate aggr='add', GNN.py:134) as the native forward runs
    it -- cgr_segment_sum over the dst-sorted edge rows [E, H] into [N, H] -- and its backward
    twin (rows gathered through the src permutation), each timed as `reps` back-to-back launches
    between two HIP events on the launch stream (a single ~8 us launch between events also
    times the event/dispatch gap).  Inputs are HBM-resident, sized like the bench batch.

    Two cache states: "warm" re-reads one input, which (24.6 MB at cfg2) stays in the 256 MB
    Infinity Cache between launches, so it measures the cache more than HBM; "cold" rotates over
    `cold_copies` distinct inputs and outputs (> 256 MB per rotation: 24 x 36.9 MB = 886 MB at
    cfg2), so every launch streams from HBM.  `which`: only these (name, state) pairs (the PMC
    tool, tools/scatter_pmc.py)."""
    from cgr_mpnn_3D._amd import native

    lib = native.load()
    E = edge_index.shape[1]
    src, dst = edge_index[0], edge_index[1]

    def csr(keys):
        deg = torch.bincount(keys, minlength=N)
        ptr = torch.zeros(N + 1, dtype=torch.int32, device=dev)
        ptr[1:] = torch.cumsum(deg, 0).to(torch.int32)
        return ptr

    ptr_dst = csr(dst)
    ptr_src = csr(src)
    perm_src = torch.argsort(src, stable=True).to(torch.int32)
    stream = torch.cuda.current_stream(dev)
    res = {}
    for state in ("warm", "cold"):
        copies = 1 if state == "warm" else max(1, cold_copies)
        if which is not None and not any(w[1] == state for w in which):
            continue
        vals = [torch.randn(E, H, device=dev) for _ in range(copies)]
        outs = [torch.empty(N, H, device=dev) for _ in range(copies)]
        for name, idx, ptr in (("segsum_dst_fwd", None, ptr_dst),
                               ("segsum_src_bwd", perm_src, ptr_src)):
            if which is not None and (name, state) not in which:
                continue

            def launch(i):
                native.check(lib.cgr_segment_sum(native.ptr(vals[i % copies]), H,
                                                 native.ptr(idx), native.ptr(ptr), N, H,
                                                 native.ptr(outs[i % copies]), H,
                                                 stream.cuda_stream))
            for i in range(5):
                launch(i)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(stream)
            for i in range(reps):
                launch(5 + i)
            e1.record(stream)
            e1.synchronize()
            us = e0.elapsed_time(e1) * 1e3 / reps
            nbytes = 4.0 * (E * H + N * H) + 4.0 * (N + 1) + (4.0 * E if idx is not None else 0.0)
            res[(name, state)] = {
                "kernel": name, "bound": "hbm", "achieved": round(nbytes / us / 1e3, 2),
                "peak": HBM_PEAK_GBS, "unit": "GB/s",
                "frac": round(nbytes / us / 1e3 / HBM_PEAK_GBS, 4),
                "algorithmic_bytes_per_launch": nbytes, "avg_launch_us": round(us, 3),
                "cache_state": state,
                "timing": f"{reps} back-to-back cgr_segment_sum launches between HIP events on the "
                          f"launch stream, E={E} rows x H={H} -> N={N}"
                          + (f", rotating over {copies} distinct input/output pairs "
                             f"({copies * nbytes / 1e6:.0f} MB per rotation > the 256 MB "
                             f"Infinity Cache)" if copies > 1 else
                             ", one input re-read (Infinity-Cache resident)")}
        if which is None:
            # streaming reference at the same cache state and byte shape: out = v[:E/2] +
            # v[E/2:] (torch's vectorised elementwise add: reads E rows, writes E/2 = N rows at
            # the bench shapes) -- what a plain coalesced stream of these bytes achieves on this
            # box, the practical ceiling the segmented sum is compared against
            h = E // 2
            refo = [torch.empty(h, H, device=dev) for _ in range(copies)]
            with torch.cuda.stream(stream):
                for i in range(5):
                    torch.add(vals[i % copies][:h], vals[i % copies][h:2 * h],
                              out=refo[i % copies])
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record(stream)
                for i in range(reps):
                    k = (5 + i) % copies
                    torch.add(vals[k][:h], vals[k][h:2 * h], out=refo[k])
                e1.record(stream)
            e1.synchronize()
            us = e0.elapsed_time(e1) * 1e3 / reps
            rb = 4.0 * (2 * h * H + h * H)
            ref = {"kernel": "torch.add(v[:E/2], v[E/2:]) (2 reads, 1 write per output row)",
                   "achieved": round(rb / us / 1e3, 2), "unit": "GB/s", "avg_launch_us": round(us, 3),
                   "bytes_per_launch": rb}
            for name in ("segsum_dst_fwd", "segsum_src_bwd"):
                if (name, state) in res:
                    res[(name, state)]["streaming_reference"] = ref
                    res[(name, state)]["frac_of_streaming_reference"] = round(
                        res[(name, state)]["achieved"] / ref["achieved"], 4)
            del refo
        del vals, outs
    return res


def collate_measurement(cfgname, dev, store_graphs=4096, reps=50):
    """§8(f) rank 1: on-device collation (cgr_collate) of one bench-sized batch of random graph
    ids out of a device-resident store, vs the PyG collation restated in numpy on the host
    (oracle/collate_numpy.py, the CPU baseline of this leg)."""
    import numpy as np

    from cgr_mpnn_3D._amd import native
    from cgr_mpnn_3D._amd.data import GraphStore
    from cgr_mpnn_3D._amd.synth import CONFIGS, make_batch
    from oracle import collate_numpy as oc

    c = CONFIGS[cfgname]
    allb = make_batch(store_graphs, c["n_atoms"], c["n_bonds"], c["n_mace"], seed=4321)
    store = GraphStore.from_batch(allb, dev)
    rng = np.random.default_rng(0)
    ids = rng.integers(0, store_graphs, size=c["num_graphs"])
    B = ids.size
    N, E = store.batch_sizes(ids)
    lib = native.load()
    gid = torch.from_numpy(ids).to(dev)
    x = torch.empty((N, store.F), device=dev)
    ei = torch.empty((2, E), dtype=torch.int64, device=dev)
    ea = torch.empty((E, store.Fe), device=dev)
    bt = torch.empty(N, dtype=torch.int64, device=dev)
    ptr = torch.empty(B + 1, dtype=torch.int64, device=dev)
    y = torch.empty(B, device=dev)
    stream = torch.cuda.current_stream(dev)

    def launch():
        native.check(lib.cgr_collate(
            native.ptr(gid), B, native.ptr(store.node_ptr), native.ptr(store.edge_ptr),
            native.ptr(store.x), store.F, native.ptr(store.edge_index),
            int(store.edge_index.shape[1]), native.ptr(store.edge_attr), store.Fe,
            native.ptr(store.y), native.ptr(x), native.ptr(ei), E, native.ptr(ea), native.ptr(bt),
            native.ptr(ptr), native.ptr(y), stream.cuda_stream))

    for _ in range(5):
        launch()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(stream)
    for _ in range(reps):
        launch()
    e1.record(stream)
    e1.synchronize()
    us = e0.elapsed_time(e1) * 1e3 / reps
    # algorithmic bytes: read + write of x, edge_attr, edge_index, write batch/ptr/y, read ids/ptrs
    nbytes = 2.0 * 4 * (N * store.F + E * store.Fe) + 2.0 * 8 * 2 * E + 8.0 * N + 8 * (B + 1) \
        + 4.0 * B + 8.0 * 3 * B
    # end-to-end GraphStore.collate (host ids -> device batch, allocation, H2D of the ids)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(20):
        store.collate(ids)
    torch.cuda.synchronize()
    call_us = (time.perf_counter() - t0) / 20 * 1e6
    # CPU baseline: numpy restatement of Batch.from_data_list for the same ids
    arrays = (allb.x, allb.edge_index, allb.edge_attr, allb.y, allb.ptr, store.edge_ptr_h)
    n_cpu, t0 = 0, time.perf_counter()
    while time.perf_counter() - t0 < 2.0:
        oc.collate(ids, *arrays)
        n_cpu += 1
    cpu_s = (time.perf_counter() - t0) / n_cpu
    return {"kernel": "cgr_collate", "bound": "hbm", "avg_launch_us": round(us, 3),
            "achieved": round(nbytes / us / 1e3, 2), "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": round(nbytes / us / 1e3 / HBM_PEAK_GBS, 4),
            "algorithmic_bytes_per_launch": nbytes,
            "reactions_per_s": round(B / (us * 1e-6), 1),
            "graphstore_collate_call_us": round(call_us, 1),
            "cpu_baseline": {"value": round(B / cpu_s, 1), "unit": "reactions/s", "cores": 1,
                             "kind": "port",
                             "sample": f"{n_cpu} numpy Batch.from_data_list restatements of "
                                       f"{B} graphs (oracle/collate_numpy.py), 1 thread"},
            "store": f"{store_graphs} {cfgname}-shaped reactions resident "
                     f"({store.x.numel() * 4 / 1e9:.2f} GB of x)",
            "timing": f"{reps} back-to-back launches between HIP events"}


def inference_measurement(model, data, B, dev, steps=50):
    """§8(f) rank 3: eval-mode forward only (dropout off, no autograd) on the bench batch,
    captured into a HIP graph like the training step; reactions/s."""
    was = model.training
    model.eval()
    try:
        with torch.no_grad():
            s = torch.cuda.Stream()
            s.wait_stream(torch.cuda.current_stream())
            with torch.cuda.stream(s):
                for _ in range(3):
                    model(data)
            torch.cuda.current_stream().wait_stream(s)
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g):
                model(data)
            for _ in range(5):
                g.replay()
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(steps):
                g.replay()
            torch.cuda.synchronize()
            el = time.perf_counter() - t0
    finally:
        model.train(was)
    return {"metric": "reactions/s (eval forward, batched)", "value": round(B * steps / el, 1),
            "ms_per_batch": round(el / steps * 1e3, 4), "batch": B, "graph_captured": True}


def single_reaction_measurement(model, cfgname, dev, calls=300, prof_calls=20):
    """§8(f) rank 3, the reference's own inference call pattern: ONE reaction per forward, eval
    mode, under no_grad -- test.py:85-113 (DataLoader batch_size 1: a one-graph Batch) and
    cli_tool/activation_energy_predictor.py:72-76 (a single Data, batch=None).  Per pattern:
    the median latency of `model(data)` + synchronize (the CLI reads each prediction), the host
    time to enqueue one call (calls issued back to back), and the device time of one call's
    kernels (library HIP events per kernel class, summed)."""
    import numpy as np

    from cgr_mpnn_3D._amd import native
    from cgr_mpnn_3D._amd.synth import CONFIGS, TorchBatch, make_batch

    c = CONFIGS[cfgname]
    b = make_batch(1, c["n_atoms"], c["n_bonds"], c["n_mace"], seed=4242)
    x = torch.from_numpy(b.x).to(dev)
    ei = torch.from_numpy(b.edge_index).to(dev)
    ea = torch.from_numpy(b.edge_attr).to(dev)
    pats = {"batch_none_cli": TorchBatch(x, ei, ea, None),
            "one_graph_batch_test_py": TorchBatch(x, ei, ea, torch.from_numpy(b.batch).to(dev),
                                                  torch.from_numpy(b.ptr).to(dev))}
    lib = native.load()
    was = model.training
    model.eval()
    out = {"graph": f"one {cfgname}-shaped reaction: N={x.shape[0]} atoms, E={ei.shape[1]} "
                    f"directed edges, F={x.shape[1]}"}
    try:
        with torch.no_grad():
            for name, d in pats.items():
                for _ in range(20):
                    model(d)
                torch.cuda.synchronize()
                lat = []
                for _ in range(calls):
                    t0 = time.perf_counter()
                    model(d)
                    torch.cuda.synchronize()
                    lat.append(time.perf_counter() - t0)
                t0 = time.perf_counter()
                for _ in range(100):
                    model(d)
                host = (time.perf_counter() - t0) / 100
                torch.cuda.synchronize()
                lib.cgr_profile_reset()
                lib.cgr_profile_enable(1)
                for _ in range(prof_calls):
                    model(d)
                torch.cuda.synchronize()
                lib.cgr_profile_enable(0)
                rep = native.profile_report()
                dev_ms = sum(t for _, t in rep.values()) / prof_calls
                launches = sum(n for n, _ in rep.values()) / prof_calls
                out[name] = {"latency_us_median": round(float(np.median(lat)) * 1e6, 1),
                             "latency_us_p90": round(float(np.percentile(lat, 90)) * 1e6, 1),
                             "host_enqueue_us": round(host * 1e6, 1),
                             "device_us": round(dev_ms * 1e3, 1),
                             "kernel_classes_per_call": round(launches, 1),
                             "device_us_by_class": {k: round(t / prof_calls * 1e3, 2)
                                                    for k, (_, t) in sorted(rep.items())},
                             "reactions_per_s": round(1.0 / float(np.median(lat)), 1)}
    finally:
        model.train(was)
    out["single_reaction_us"] = out["batch_none_cli"]["latency_us_median"]
    return out


# ------------------------------------------------------------------------------------------------
def host_cpu_info():
    """What the CPU baseline ran on: the CPU model, the machine's physical cores and logical
    CPUs, the CPUs this process may run on, and the torch intra-op threads the baseline used
    (`cores` of the cpu_baseline object = those threads)."""
    model = None
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    model = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    try:
        import psutil

        phys, logical = psutil.cpu_count(logical=False), psutil.cpu_count(logical=True)
    except Exception:  # noqa: BLE001
        phys, logical = None, os.cpu_count()
    try:
        allowed = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        allowed = None
    quota = None  # cgroup v2 CPU bandwidth limit of this process ("max" = none), in CPUs
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        quota = None if q == "max" else round(int(q) / int(per), 2)
    except (OSError, ValueError):
        pass
    return {"cpu_model": model, "machine_physical_cores": phys, "machine_logical_cpus": logical,
            "process_allowed_cpus": allowed, "cgroup_cpu_quota": quota,
            "torch_threads": torch.get_num_threads(),
            "omp_num_threads_env": os.environ.get("OMP_NUM_THREADS")}


def host_physical_cores():
    """Physical cores this process may run on: the CPUs in its affinity mask scaled by the
    machine's physical / logical ratio (SMT siblings are not extra cores)."""
    info = host_cpu_info()
    allowed = info["process_allowed_cpus"] or info["machine_logical_cpus"] or 1
    phys, logical = info["machine_physical_cores"], info["machine_logical_cpus"]
    if phys and logical:
        return max(1, round(allowed * phys / logical))
    return allowed  # (a cgroup CPU quota, if any, is recorded by host_cpu_info, not applied)


def cpu_baseline_both(cfgname, seconds, dropout):
    """the CPU baseline on the whole host (torch threads = the physical cores this
    process may use) and, beside it, at the torch default (OMP_NUM_THREADS, 16 on the GPU boxes);
    the line's `cpu_baseline` is the faster of the two, the other is kept under `alternative`."""
    default_threads = torch.get_num_threads()
    full = host_physical_cores()
    runs = []
    try:
        for t in dict.fromkeys([full, default_threads]):
            torch.set_num_threads(t)
            runs.append(cpu_baseline(cfgname, seconds, dropout))
    finally:
        torch.set_num_threads(default_threads)
    best = max(runs, key=lambda r: r["value"])
    others = [r for r in runs if r is not best]
    if others:
        best = dict(best, alternative={k: others[0][k] for k in ("value", "cores", "sample")})
    best["threads_rule"] = (f"timed at {full} threads (the physical cores this process may use) "
                            f"and at the torch default {default_threads}; the faster is the "
                            f"baseline")
    return best


def cpu_baseline(cfgname, seconds, dropout):
    """Reference CPU path (oracle/dmpnn_torch.py: the reference ATen op sequence incl. its dead
    readout GEMM) on this host's cores: same batch shape, MSE(sum) + backward + Adam(amsgrad)."""
    from cgr_mpnn_3D._amd.synth import CONFIGS, make_batch
    from oracle.dmpnn_torch import TorchRestatement, random_state_dict

    c = CONFIGS[cfgname]
    b = make_batch(c["num_graphs"], c["n_atoms"], c["n_bonds"], c["n_mace"], seed=1234)
    F_ = b.x.shape[1]
    sd = random_state_dict(F_, 14, c["hidden"], c["depth"], c["learnable_skip"], seed=0)
    m = TorchRestatement(sd, c["depth"], learnable_skip=c["learnable_skip"],
                         dropout_ps=[dropout] * c["depth"])
    m.train()
    opt = torch.optim.Adam(m.parameters(), lr=1e-3, amsgrad=True)
    x = torch.from_numpy(b.x)
    ei = torch.from_numpy(b.edge_index)
    ea = torch.from_numpy(b.edge_attr)
    bt = torch.from_numpy(b.batch)
    y = torch.from_numpy(b.y)
    loss_fn = torch.nn.MSELoss(reduction="sum")

    def step():
        opt.zero_grad()
        loss = loss_fn(m(x, ei, ea, bt, b.num_graphs), y)
        loss.backward()
        opt.step()

    for _ in range(2):
        step()
    n = 0
    t0 = time.perf_counter()
    while True:
        step()
        n += 1
        el = time.perf_counter() - t0
        if el >= seconds or n >= 200:
            break
    return {"value": round(n * b.num_graphs / el, 2), "unit": "reactions/s",
            "cores": torch.get_num_threads(), "kind": "port", "host": host_cpu_info(),
            "sample": f"{n} training steps of the {cfgname} batch ({b.num_graphs} reactions, "
                      f"fwd+MSE+bwd+Adam) with the torch-CPU restatement of the reference op "
                      f"sequence, {el:.1f} s, torch {torch.__version__}, "
                      f"{torch.get_num_threads()} threads"}


def _free_port() -> int:
    import socket

    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def spawn_ranks(n: int, cmd: list[str], env: dict | None = None, poll_s: float = 0.2) -> int:
    """Run `cmd` as `n` fresh child processes, one per rank, with RANK / LOCAL_RANK / WORLD_SIZE /
    MASTER_ADDR (127.0.0.1) / MASTER_PORT set -- what `torch.distributed.run --nnodes=1
    --nproc-per-node n` would set.  The caller must not have touched the GPU: the children are
    started with subprocess (no exec), inherit stdout / stderr (rank 0's JSON line goes straight
    through), and are waited for.  If one child fails, the others are terminated (then killed)
    by PID so that a rank blocked in a collective does not hang the job.  Returns the first
    non-zero exit status (negative = the signal a child died of), else 0."""
    import subprocess

    base = dict(os.environ if env is None else env)
    base.setdefault("MASTER_ADDR", "127.0.0.1")
    base.setdefault("MASTER_PORT", str(_free_port()))
    base["WORLD_SIZE"] = str(n)
    base["LOCAL_WORLD_SIZE"] = str(n)
    base["CGR_BENCH_SPAWNED"] = "1"
    procs = []
    for r in range(n):
        e = dict(base, RANK=str(r), LOCAL_RANK=str(r), GROUP_RANK="0")
        procs.append(subprocess.Popen(cmd, env=e))
    rc = 0
    try:
        while True:
            alive = False
            for r, p in enumerate(procs):
                s = p.poll()
                if s is None:
                    alive = True
                elif s != 0 and rc == 0:
                    rc = s
                    log(f"[bench] rank {r} exited with status {s}; stopping the other ranks")
            if rc != 0 or not alive:
                break
            time.sleep(poll_s)
    finally:
        for p in procs:
            if p.poll() is None:
                p.terminate()
        for p in procs:
            try:
                p.wait(timeout=20)
            except subprocess.TimeoutExpired:
                p.kill()
                p.wait()
    return rc


def main():
    args = parse()
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        # no outside launcher: start the N ranks here, before anything touches the GPU
        sys.exit(spawn_ranks(args.gpus, [sys.executable, "-u", os.path.abspath(__file__)]
                             + sys.argv[1:]))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise SystemExit(f"--gpus {args.gpus} but WORLD_SIZE={world}")
    if args.graph < 0:
        # N > 1 too: the RCCL all-reduce of the gradient bucket is captured with the step
        # (rehearsed on one GPU with --force-dist 1)
        args.graph = 1
    ordinal = local % max(1, torch.cuda.device_count())  # == local on a full node
    torch.cuda.set_device(ordinal)
    dev = torch.device("cuda", ordinal)
    distributed = world > 1 or bool(args.force_dist)
    if distributed:
        # an abort on a runtime thread (RCCL / HIP / c10d) prints its native stack
        from cgr_mpnn_3D._amd import native as _native

        _native.load().cgr_debug_abort_backtrace(1)
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", "29511")
        os.environ.setdefault("RANK", str(rank))
        os.environ.setdefault("WORLD_SIZE", str(world))
        if args.dist_backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group("gloo")

    from cgr_mpnn_3D._amd import native
    from cgr_mpnn_3D._amd.ddp import install_grad_allreduce
    from cgr_mpnn_3D._amd.synth import CONFIGS, make_batch
    from cgr_mpnn_3D.models.GNN import GNN

    c = CONFIGS[args.config]
    D, H = c["depth"], c["hidden"]
    b = make_batch(c["num_graphs"], c["n_atoms"], c["n_bonds"], c["n_mace"], seed=1234 + rank)
    data = b.to_torch(dev)
    N, E, B = b.x.shape[0], b.edge_index.shape[1], b.num_graphs
    F_ = b.x.shape[1]
    torch.manual_seed(0)
    model = GNN(F_, 14, depth=D, hidden_sizes=[H] * D, dropout_ps=[args.dropout] * D,
                use_learnable_skip=c["learnable_skip"]).to(dev)
    model.train()
    if distributed:
        install_grad_allreduce(model)
    if args.optimizer == "fused":
        from cgr_mpnn_3D._amd.optim import FusedAdam

        opt = FusedAdam(model.parameters(), lr=1e-3, amsgrad=True)
    else:
        opt = torch.optim.Adam(model.parameters(), lr=1e-3, amsgrad=True,
                               capturable=bool(args.graph))
    if args.loss == "fused":
        from cgr_mpnn_3D._amd.loss import MSELoss

        loss_fn = MSELoss(reduction="sum")  # native, one launch each way (train.py:120's loss)
    else:
        loss_fn = torch.nn.MSELoss(reduction="sum")

    def step():
        opt.zero_grad(set_to_none=True)
        loss = loss_fn(model(data), data.y)
        loss.backward()
        opt.step()
        return loss

    # warmup (eager), then optional graph capture of the whole step
    log(f"[bench] rank {rank}/{world} {args.config}: N={N} E={E} B={B} F={F_} H={H} D={D}")
    for _ in range(max(3, args.warmup)):
        step()
    torch.cuda.synchronize()
    run = step
    g = None
    if args.graph and distributed and args.dist_backend != "nccl":
        args.graph = 0  # a gloo collective cannot be recorded into a HIP graph (host copies)
    capture_note = None
    if args.graph:
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            for _ in range(3):
                step()
        torch.cuda.current_stream().wait_stream(s)
        ok = 1
        try:
            g = torch.cuda.CUDAGraph()
            # thread-local capture: the c10d / RCCL watchdog thread queries its own events while
            # this thread captures, which a global-mode capture treats as an error (seen once on
            # the RCCL world-1 rehearsal: "operation not permitted when stream is capturing")
            with torch.cuda.graph(g, capture_error_mode="thread_local" if distributed
                                  else "global"):
                step()
        except Exception as exc:  # noqa: BLE001
            # a capture the runtime refuses (e.g. a collective RCCL cannot record at this world
            # size) must not end the scaling run: every rank then times the eager step
            log(f"[bench] rank {rank}: step capture failed ({type(exc).__name__}: {exc}); "
                f"timing the eager step")
            g, ok = None, 0
            torch.cuda.synchronize()
        if world > 1:  # all ranks replay, or none does (a lone replayer would hang the others)
            flag = torch.tensor([ok], device=dev, dtype=torch.int32)
            dist.all_reduce(flag, op=dist.ReduceOp.MIN)
            ok = int(flag.item())
        if ok:
            run = g.replay
        else:
            g = None
            args.graph = 0
            capture_note = "step capture failed on at least one rank; eager step timed"
        for _ in range(args.warmup):
            run()
        torch.cuda.synchronize()
    # steady state before the timed region: a freshly captured step runs
    # ~13 % slower for its first ~40 replays (0.85 -> 0.75 ms at cfg2, per-step stamps,
    # tools/clock_gap.py) whatever W is, so the untimed warmup continues until the device has
    # spent --min-warmup-ms in back-to-back steps.  The count is agreed across ranks (every
    # replay holds collectives when N > 1).
    warm_extra = 0
    if args.min_warmup_ms > 0:
        torch.cuda.synchronize()
        t_w = time.perf_counter()
        for _ in range(3):
            run()
        torch.cuda.synchronize()
        per = (time.perf_counter() - t_w) / 3
        warm_extra = max(0, int(args.min_warmup_ms * 1e-3 / max(per, 1e-6)) - 3)
        warm_extra = min(warm_extra, 20000)
        if world > 1:
            t = torch.tensor([warm_extra], device=dev, dtype=torch.int64)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            warm_extra = int(t.item())
        for i in range(warm_extra):
            run()
            if (i + 1) % 50 == 0:
                torch.cuda.synchronize()  # keep the host within 50 steps of the device
        torch.cuda.synchronize()
        warm_extra += 3

    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(args.steps):
        run()
        if rank == 0 and (i + 1) % max(1, args.steps // 5) == 0:
            log(f"[bench] step {i + 1}/{args.steps}")
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    el = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([el], device=dev, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        el = float(t.item())
    ms = el / args.steps * 1e3
    value = world * B * args.steps / el

    diag = None
    if args.diag_blocks > 0:
        # more blocks of K steps straight after the timed one, each timed like
        # it (host clock, device synchronised) plus a HIP event before every step on the launch
        # stream -- whether the first K steps after a short warmup run slower than later ones
        diag = []
        stream = torch.cuda.current_stream(dev)
        for _ in range(args.diag_blocks):
            evs = [torch.cuda.Event(enable_timing=True) for _ in range(args.steps + 1)]
            torch.cuda.synchronize()
            t1 = time.perf_counter()
            for i in range(args.steps):
                evs[i].record(stream)
                run()
            evs[-1].record(stream)
            torch.cuda.synchronize()
            bl = time.perf_counter() - t1
            st = [evs[i].elapsed_time(evs[i + 1]) for i in range(args.steps)]
            diag.append({"ms_per_step": round(bl / args.steps * 1e3, 4),
                         "event_ms_per_step": round(sum(st) / len(st), 4),
                         "event_ms_first_last": [round(st[0], 4), round(st[-1], 4)],
                         "event_ms_min_max": [round(min(st), 4), round(max(st), 4)]})

    # per-kernel-class device time with HIP events on the launch stream (eager, instrumented)
    lib = native.load()
    roof = None
    roof_scatter = None
    roof_all = {}
    breakdown = {}
    # gloo rehearsal (several ranks on one GPU, host-staged collectives): the instrumented pass
    # would time kernels queued behind other ranks' work and gloo's host copies -- meaningless
    # per-kernel durations, so the line carries no roofline then
    gloo_rehearsal = distributed and args.dist_backend == "gloo"
    if args.profile_steps > 0 and not gloo_rehearsal:
        lib.cgr_profile_reset()
        lib.cgr_profile_enable(1)
        for _ in range(args.profile_steps):
            step()
        torch.cuda.synchronize()
        lib.cgr_profile_enable(0)
        rep = native.profile_report()
        work = algorithmic_work(N, E, B, F_, 14, H, D)
        traffic = {}
        if os.path.exists(args.traffic_json):
            try:
                traffic = json.load(open(args.traffic_json)).get(args.config, {})
            except Exception:  # noqa: BLE001
                traffic = {}

        def base(name):  # "<class>[f32]" / "[tnr]": the fp32 fallback family of a class
            return name.split("[")[0]

        def hbm(name):
            t = traffic.get(base(name))
            return None if t is None else t.get("hbm_bytes_per_launch")

        for name, (cnt, tot) in rep.items():
            breakdown[name] = {"launches_per_step": cnt / args.profile_steps,
                               "ms_per_step": round(tot / args.profile_steps, 5)}
        work.update({k: work[base(k)] for k in rep if k not in work and base(k) in work})
        cands = [k for k in rep if k in work]
        if cands:
            dom = max(cands, key=lambda k: rep[k][1])
            roof = roofline_entry(dom, work[dom], rep[dom][0], rep[dom][1], hbm(dom))
        sc = scatter_add_roofline(data.edge_index, N, H, dev)
        # the headline is the HBM-streaming (cold) form; the cache-resident one is reported beside
        roof_scatter = sc[("segsum_dst_fwd", "cold")]
        roof_scatter["traffic"] = hbm("segsum_dst_fwd_cold")
        roof_scatter["warm_cache"] = dict(sc[("segsum_dst_fwd", "warm")],
                                          traffic=hbm("segsum_dst_fwd"))
        roof_scatter["backward_gather_twin"] = dict(sc[("segsum_src_bwd", "cold")],
                                                    traffic=hbm("segsum_src_twin_cold"))
        if args.config == "cfg2":
            # the same kernel on cfg4's edge set (200-atom reactions, E = 204,800; 491 MB per
            # launch, beyond the Infinity Cache with two rotating copies), same box, same run
            from cgr_mpnn_3D._amd.synth import CONFIGS as _C, make_batch as _mb

            c4 = _C["cfg4"]
            b4 = _mb(c4["num_graphs"], c4["n_atoms"], c4["n_bonds"], 0, seed=1234)
            sc4 = scatter_add_roofline(torch.from_numpy(b4.edge_index).to(dev), b4.x.shape[0], H,
                                       dev, reps=20, cold_copies=2,
                                       which=[("segsum_dst_fwd", "cold")])
            roof_scatter["at_cfg4_edge_set"] = sc4[("segsum_dst_fwd", "cold")]
            del b4, sc4
        # inside the step: the forward's scatter-adds run in the layer GEMM's epilogue (no
        # kernel of their own); the backward's Gs = segsum_src(dpre0) is a standalone one
        if "segsum_src_bwd" in rep:
            cnt_s, tot_s = rep["segsum_src_bwd"]
            roof_scatter["in_step_backward_gather"] = roofline_entry(
                "segsum_src_bwd", work["segsum_src_bwd"], cnt_s, tot_s, hbm("segsum_src_bwd"))
        roof_all = {k: roofline_entry(k, work[k], rep[k][0], rep[k][1], hbm(k))["frac"]
                    for k in cands}

    coll = None
    if rank == 0 and world == 1 and args.collate_bench:
        coll = collate_measurement(args.config, dev)
    infer = None
    if rank == 0 and world == 1 and args.infer_bench:
        infer = inference_measurement(model, data, B, dev)
        infer["single_reaction"] = single_reaction_measurement(model, args.config, dev)
        if args.profile_steps > 0:  # per-class device time of the forward-only path
            was = model.training
            model.eval()
            lib.cgr_profile_reset()
            lib.cgr_profile_enable(1)
            with torch.no_grad():
                for _ in range(args.profile_steps):
                    model(data)
            torch.cuda.synchronize()
            lib.cgr_profile_enable(0)
            model.train(was)
            irep = native.profile_report()
            work = algorithmic_work(N, E, B, F_, 14, H, D)
            ic = [k for k in irep if k in work]
            if ic:
                dom = max(ic, key=lambda k: irep[k][1])
                infer["roofline"] = roofline_entry(dom, work[dom], irep[dom][0], irep[dom][1], None)
                infer["kernel_breakdown"] = {
                    k: {"launches_per_batch": cnt / args.profile_steps,
                        "ms_per_batch": round(tot / args.profile_steps, 5)}
                    for k, (cnt, tot) in irep.items()}

    cpu = None
    if rank == 0 and world == 1 and args.cpu_baseline:
        log("[bench] timing the CPU baseline (reference op sequence, torch CPU) ...")
        cpu = cpu_baseline_both(args.config, args.cpu_seconds, args.dropout)

    if rank == 0:
        out = {
            "metric": METRIC, "value": round(value, 2), "unit": "reactions/s", "n_gpus": world,
            "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(ms, 4),
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None,
            "dtype": "bf16-split/fp32-acc",
            "precision": "fp32 data; GEMMs on the bf16 matrix cores from exact bf16 pieces of the "
                         "fp32 operands (NT: 3 pieces, 6 products, ~fp32; weight-gradient TN: 2 "
                         "pieces, 3 products, >=16-bit operand mantissa), fp32 accumulation; "
                         "everything else fp32 (DESIGN.md §2)",
            "data": "synthetic T1x-shaped batches (seeded generator, HBM-resident), random-init "
                    "weights",
            "config": {
                "workload": f"{args.config}: CGR-MPNN-3D depth={D} hidden={H}, {B} reactions/GPU "
                            f"({c['n_atoms']} atoms, {2 * c['n_bonds']} directed edges each), "
                            f"F={F_} (78 CGR + {c['n_mace']} MACE), Fe=14, ReLU, dropout {args.dropout}; step "
                            f"= fwd + MSELoss(sum, {'native' if args.loss == 'fused' else 'torch'}) + bwd + grad all-reduce (N>1) + "
                            f"Adam(amsgrad, {'fused native' if args.optimizer == 'fused' else 'torch foreach'})"
                            + (", HIP-graph captured" if args.graph else ""),
                "global_batch": world * B, "parallelism": f"dp{world}"},
            "roofline": roof, "roofline_scatter_add": roof_scatter,
            "roofline_note": ("omitted: gloo rehearsal (ranks share one GPU; the instrumented "
                              "pass would time other ranks' work and gloo's host copies)")
            if gloo_rehearsal else None,
            "roofline_frac_by_class": roof_all, "kernel_breakdown": breakdown,
            "cpu_baseline": cpu,
        }
        out["warmup_steady"] = {"extra_untimed_steps": warm_extra,
                                "min_warmup_ms": args.min_warmup_ms,
                                "why": "a new captured step runs slower for its first ~40 "
                                       "replays; the untimed warmup runs W steps and then until "
                                       "min_warmup_ms of steps (DESIGN.md §9)"}
        if diag is not None:
            out["diag_blocks"] = diag
        if capture_note:
            out["capture_note"] = capture_note
        if os.environ.get("CGR_BENCH_SPAWNED") == "1":
            out["launcher"] = "bench.py spawned its own ranks (no torch.distributed.run)"
        if coll is not None:
            out["collate"] = coll
        if infer is not None:
            out["inference"] = infer
        if cpu:
            out["speedup_vs_cpu_baseline"] = round(value / cpu["value"], 2)
        print(json.dumps(out), flush=True)
    if distributed:
        # captured graph (it recorded the per-bucket collectives) first, then the communicator
        # (ddp.teardown explains the order)
        from cgr_mpnn_3D._amd.ddp import teardown

        run = g = None  # noqa: F841
        teardown(model, graphs_released=True)


if __name__ == "__main__":
    main()
