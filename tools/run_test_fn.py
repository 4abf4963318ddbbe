"""Run one test function of tests/ outside pytest (debugging): run_test_fn.py MODULE FUNC"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "tests"))
import conftest  # noqa: E402,F401  (sets sys.path like pytest does)
import importlib  # noqa: E402

import torch  # noqa: E402

mod = importlib.import_module(sys.argv[1])
fn = getattr(mod, sys.argv[2])
print("[run_test_fn] calling", sys.argv[2], flush=True)
fn(torch.device("cuda:0")) if fn.__code__.co_argcount else fn()
print("[run_test_fn] ok", flush=True)
