"""HIP-kernel-backed operations (CPU tensors use the PyTorch reference paths)."""
from . import random
