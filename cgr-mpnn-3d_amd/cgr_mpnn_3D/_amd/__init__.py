"""Native (HIP/gfx950) backend of cgr_mpnn_3D: ctypes binding, autograd bridge, DDP helpers."""
