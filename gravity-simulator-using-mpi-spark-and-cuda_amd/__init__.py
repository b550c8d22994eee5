"""gravsim — MI355X-native direct-sum N-body gravity simulator.

Capabilities of the MPI/Spark/CUDA reference (pdpatel13/Gravity-Simulator-using-MPI-Spark-and-CUDA:
cuda.cu, mpi.c, pyspark.py), re-designed for AMD Instinct MI355X (gfx950):

* `models`   — initial-condition families (Sun/Earth/Mars + random bodies, random cube,
               Plummer sphere, Kepler two-body), counter-based and rank-count independent.
* `ops`      — force/step operators: hand-written HIP gfx950 kernels (libgravsim_hip.so),
               the native C++ CPU engine (libgravsim_cpu.so) and the NumPy fp64 oracle.
* `parallel` — canonical body decomposition, process-group bootstrap, RCCL/gloo exchange,
               virtual ranks.
* `runtime`  — the Simulation driver (step loop, NaN guard, checkpoints, trajectories).
* `utils`    — reference-format logs and dumps (mpi.c / pyspark.py / cuda.cu), binary
               checkpoints, JSON metrics, timing.

Import as `import gravsim` from the repository root (gravsim.py is the import shim).
"""
from .config import SimConfig, G_SI  # noqa: F401

__version__ = "0.1.0"


def __getattr__(name):  # lazy: keep `import gravsim` light (no torch / native load)
    if name in ("GravitySimulator", "SparkGravitySimulator", "Particle", "create_solar_system",
                "generate_random_particles"):
        from . import api

        return getattr(api, name)
    if name == "Simulation":
        from .runtime.simulation import Simulation

        return Simulation
    raise AttributeError(name)


__all__ = ["SimConfig", "G_SI", "Simulation", "GravitySimulator", "SparkGravitySimulator",
           "Particle", "create_solar_system", "generate_random_particles", "__version__"]
