"""Parallel execution: canonical decomposition, process bootstrap, exchanges, virtual ranks.

Strategy: body ("row") decomposition with replicated positions — each
rank owns a contiguous slice of bodies, sums their full force rows against all N, integrates
them, and all-gathers positions every step (mpi.c:184-231 analogue). On MI355X the exchange
is an in-place RCCL all-gather over xGMI overlapped with the rank-local j-chunks.
"""
from .partition import Layout, layout, auto_chunk, mpi_block  # noqa: F401
from .comm import DistInfo, env_info, init, shutdown, barrier  # noqa: F401
