"""Synthetic trace generation and trace file formats."""
from .format import read_kernel_binary, write_kernel_binary, write_kernel_text, write_kernelslist  # noqa: F401
