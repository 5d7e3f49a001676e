"""regcn_amd — MI355X-native hot path of RE-GCN (sgxxyyds/RE-GCN).

Host side (PyTorch-ROCm) mirroring the reference's operator interfaces for the
per-timestep relational message passing + hyperbolic scoring loop; compute in
hand-written gfx950 HIP kernels behind the C-ABI of libregcn_hip.so
(include/regcn_hip.h).  See DESIGN.md.
"""
__version__ = "0.1.0"
