import glob
import json
import os
import sys

import numpy as np
import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(REPO, "cgr-mpnn-3d_amd")
for p in (REPO, PKG):
    if p not in sys.path:
        sys.path.insert(0, p)

GOLDEN_DIR = os.path.join(REPO, "tests", "golden")

# activation name -> the callable handed to GNN(activation_fn=...); the order is the native
# cgr_activation code (include/cgr_mpnn3d.h)
ACT_NAMES = ("relu", "silu", "gelu", "tanh", "sigmoid", "elu", "leaky_relu", "softplus", "mish",
             "selu")


def act_fn(name):
    import torch
    import torch.nn.functional as F
    return {"relu": F.relu, "silu": F.silu, "gelu": F.gelu, "tanh": torch.tanh,
            "sigmoid": torch.sigmoid, "elu": F.elu, "leaky_relu": F.leaky_relu,
            "softplus": F.softplus, "mish": F.mish, "selu": F.selu}[name]


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through the HIP C-ABI)")


def golden_cases():
    out = []
    for f in sorted(glob.glob(os.path.join(GOLDEN_DIR, "*.npz"))):
        z = np.load(f, allow_pickle=False)
        if "meta" in z.files:
            out.append(os.path.basename(f)[:-4])
    return out


def load_golden(name):
    z = np.load(os.path.join(GOLDEN_DIR, name + ".npz"), allow_pickle=False)
    meta = json.loads(str(z["meta"])) if "meta" in z.files else {}
    return z, meta


@pytest.fixture(scope="session")
def cuda_device():
    import torch

    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch.device("cuda:0")
