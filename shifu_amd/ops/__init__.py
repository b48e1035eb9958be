"""Hand-written CDNA4 (gfx950) HIP kernels and their host-side launchers."""
from . import _native  # noqa: F401
