"""picotron_amd — MI355X-native (gfx950) rebuild of picotron's per-step Llama training hot path.

Kernels live in picotron_amd/csrc (HIP, C ABI in include/picotron_hip.h) and are loaded by
picotron_amd/_lib.py. torch is imported first so the library binds to torch's HIP runtime.
"""
import torch  # noqa: F401  (load torch's libamdhip64 before the kernel library)

from . import _lib  # noqa: F401

__all__ = ["_lib"]
