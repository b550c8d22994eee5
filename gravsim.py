"""Import shim: exposes the package directory `gravity-simulator-using-mpi-spark-and-cuda_amd/`
under the importable name `gravsim` (a directory name with dashes cannot be imported directly).

`import gravsim` / `python -m gravsim ...` both work from the repository root.
"""
import importlib.util
import os
import sys

_PKG_DIR = os.path.join(os.path.dirname(os.path.abspath(__file__)),
                        "gravity-simulator-using-mpi-spark-and-cuda_amd")


def _load():
    spec = importlib.util.spec_from_file_location(
        "gravsim", os.path.join(_PKG_DIR, "__init__.py"), submodule_search_locations=[_PKG_DIR])
    mod = importlib.util.module_from_spec(spec)
    sys.modules["gravsim"] = mod
    spec.loader.exec_module(mod)
    return mod


if __name__ == "__main__":
    _pkg = _load()
    from gravsim.cli import main  # noqa: E402

    sys.exit(main())
else:
    _load()
