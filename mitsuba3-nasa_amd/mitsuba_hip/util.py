"""mi.util subset on the hot path's outputs (src/python/python/util.py)."""
from .imageio import read_bitmap, write_bitmap  # noqa: F401
from .render import render, traverse  # noqa: F401
