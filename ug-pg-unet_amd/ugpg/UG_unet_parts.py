"""Alias of the reference module name UG_unet_parts (drop-in import path)."""
from .unet_parts import DoubleConv, Down, InConv, OutConv, Up  # noqa: F401
