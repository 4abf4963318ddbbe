"""Process-wide switches of the native path."""

import os

# strict: after every forward, read the graph-prep status word (one device->host sync) and raise
# on out-of-range edge indices / unsorted batch vectors, and check the reference's
# N' = max(dst) + 1 == num_nodes contract (GNN.py:106 fails with RuntimeError otherwise).
strict = os.environ.get("CGR_STRICT", "0") not in ("", "0", "false", "False")

# Called with the flat fp32 gradient bucket at the end of every native backward (before the
# per-parameter views are handed to autograd).  cgr_mpnn_3D._amd.ddp installs an RCCL
# all-reduce here.
grad_bucket_hook = None
