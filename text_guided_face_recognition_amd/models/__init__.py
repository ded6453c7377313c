"""Mirror of the reference's ``models`` package surface for the hot path."""
from . import attention, fusion_nets, losses, metrics, models  # noqa: F401
