"""Model families: initial conditions of the simulated systems, and system diagnostics."""
from .initial_conditions import (BodySet, FAMILIES, SOLAR, make, solar_random,  # noqa: F401
                                 random_cube, plummer, kepler, cold_sphere)
from .diagnostics import energy, momentum, center_of_mass  # noqa: F401
