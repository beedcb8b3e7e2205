"""zsaac — MI355X-native (gfx950 HIP) hot path of XinMing0411/zero-shot-AAC.

Host code on PyTorch-ROCm (device memory, streams, graphs, torch.distributed) calling the
hand-written CDNA4 kernels of libzsaac_hip.so through its C-ABI (include/zsaac.h).
See DESIGN.md for the path, boundary and data layout.
"""
from ._lib import ZS_BF16, ZS_F32, ZsError, build, device_arch, lib  # noqa: F401

__version__ = "0.1.0"
