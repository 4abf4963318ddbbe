"""Build record of the native library (nothing showed that the shipped .so was built
from the sources beside it).

`make` (csrc/Makefile) runs ``python3 buildinfo.py write <lib dir>/build_info.json <flags>`` right
after linking: the SHA-256 over every source the library is compiled from (csrc/*.hip, *.hpp, the
Makefile, include/*.h), the compiler's version line, the target and the flags.  ``check()``
recomputes the hash over the tree it runs in and compares (tests/test_abi.py; smoke() prints it),
so a library that is stale against its sources fails loudly instead of running silently.
"""

from __future__ import annotations

import glob
import hashlib
import json
import os
import subprocess
import sys
import time

_HERE = os.path.dirname(os.path.abspath(__file__))
PKG = os.path.dirname(os.path.dirname(_HERE))          # cgr-mpnn-3d_amd/
REPO = os.path.dirname(PKG)
CSRC = os.path.join(PKG, "csrc")
INFO = os.path.join(_HERE, "lib", "build_info.json")


def source_files() -> list[str]:
    files = []
    for pat in ("*.hip", "*.hpp", "Makefile"):
        files += glob.glob(os.path.join(CSRC, pat))
    files += glob.glob(os.path.join(REPO, "include", "*.h"))
    return sorted(files)


def source_hash() -> str:
    h = hashlib.sha256()
    for f in source_files():
        h.update(os.path.relpath(f, REPO).encode() + b"\0")
        with open(f, "rb") as fh:
            h.update(fh.read())
        h.update(b"\0")
    return h.hexdigest()


def write(path: str, flags: str = "") -> dict:
    try:
        cc = subprocess.run(["/opt/rocm/bin/hipcc", "--version"], capture_output=True,
                            text=True, timeout=60).stdout.splitlines()
        cc = next((ln for ln in cc if "clang version" in ln), cc[0] if cc else None)
    except Exception:  # noqa: BLE001
        cc = None
    info = {"sources_sha256": source_hash(), "files": len(source_files()),
            "compiler": cc, "flags": flags.strip(),
            "built_utc": time.strftime("%Y-%m-%dT%H:%M:%SZ", time.gmtime())}
    with open(path, "w") as f:
        json.dump(info, f, indent=1)
        f.write("\n")
    return info


def read(path: str = INFO) -> dict | None:
    try:
        with open(path) as f:
            return json.load(f)
    except (OSError, ValueError):
        return None


def check(path: str = INFO) -> dict:
    """The build record, with `matches_sources` = its hash equals the tree's."""
    info = read(path) or {}
    return dict(info, matches_sources=info.get("sources_sha256") == source_hash())


if __name__ == "__main__":
    if sys.argv[1] == "write":
        print(json.dumps(write(sys.argv[2], " ".join(sys.argv[3:]))))
    else:
        print(json.dumps(check()))
