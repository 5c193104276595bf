"""qdc — drop-in for the reference's Python package (src/qdc/__init__.py:1)."""
from qdc.circuit import AutoGradCircuit, VJPFunction, have_jax  # noqa: F401
