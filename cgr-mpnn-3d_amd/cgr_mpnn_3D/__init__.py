"""MI355X-native drop-in for tobjec/CGR-MPNN-3D's ``cgr_mpnn_3D`` package (hot path only).

``cgr_mpnn_3D.models.GNN`` mirrors the reference module surface; the arithmetic runs in the HIP
library ``_amd/lib/libcgr_mpnn3d.so`` (see DESIGN.md / INTEGRATION.md at the repository root).
"""
