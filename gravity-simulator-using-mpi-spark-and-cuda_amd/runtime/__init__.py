"""Runtime: execution engines (native GPU Stepper, native CPU engine, virtual ranks) and the
Simulation driver."""
from .engines import CpuEngine, HipEngine, VirtualGroup, gpu_available  # noqa: F401
from .simulation import NonFiniteError, Simulation  # noqa: F401
