"""Process-wide switches of the native path."""

import os

# strict: after every forward, read the graph-prep status word (one device->host sync) and raise
# on out-of-range edge indices / unsorted batch vectors, and check the reference's
# N' = max(dst) + 1 == num_nodes contract (GNN.py:106 fails with RuntimeError otherwise).
strict = os.environ.get("CGR_STRICT", "0") not in ("", "0", "false", "False")

# Called as hook(flat, buckets, events) after every native backward is enqueued (before the
# per-parameter views are handed to autograd): flat = the fp32 gradient buffer, buckets = its
# (start, end) ranges in the order the backward finishes them, events = their ready events (or
# None; see functional.grad_layout and ddp.GradAllReduce).  cgr_mpnn_3D._amd.ddp installs the
# RCCL all-reduce here.
grad_bucket_hook = None
