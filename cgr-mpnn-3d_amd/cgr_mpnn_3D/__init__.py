"""MI355X-native drop-in for tobjec/CGR-MPNN-3D's ``cgr_mpnn_3D`` package (hot path only).

``cgr_mpnn_3D.models.GNN`` mirrors the reference module surface; the arithmetic runs in the HIP
library ``_amd/lib/libcgr_mpnn3d.so`` (see DESIGN.md / INTEGRATION.md at the repository root).

Overlay on a reference checkout: with this package first on ``sys.path`` and
``CGR_MPNN_3D_REFERENCE`` naming the checkout (or its ``cgr_mpnn_3D`` directory), the reference's
``data``, ``training`` and ``utils`` sub-packages resolve to its files while ``models`` resolves
here (the first ``__path__`` entry that holds a name wins).
"""
import os as _os

_ref = _os.environ.get("CGR_MPNN_3D_REFERENCE")
if _ref:
    _pkg = _os.path.join(_ref, "cgr_mpnn_3D")
    _pkg = _pkg if _os.path.isdir(_pkg) else _ref
    if _os.path.abspath(_pkg) not in map(_os.path.abspath, __path__):
        __path__.append(_pkg)
