"""MI355X-native TGFR hot path: FCAM contrastive step and FCFM fusion attention.

Mirrors the reference's ``models.*`` call surface (see ``models/``); the hot
ops run as hand-written gfx950 kernels from ``lib/libtgfr_hip.so``.
"""
__version__ = "0.1.0"
