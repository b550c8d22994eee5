"""Utilities: reference-format logs/dumps, checkpoints, metrics, trajectory recording."""
from . import checkpoint, logs, metrics  # noqa: F401
