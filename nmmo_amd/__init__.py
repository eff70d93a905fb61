"""nmmo_amd — MI355X-native Neural MMO env stepper (HIP kernels behind a C-ABI)."""

from .config import Config  # noqa: F401
