"""Run csrc/tools/graph_event_probe.hip's external event-record probe on the HIP runtime a
torch process uses (the probe passed standalone, but the stepper's plan
failed with hipErrorInvalidValue at its first external record node).

Inside `python` with torch imported, torch's bundled libamdhip64.so.7 is loaded first and the
stepper's own DT_NEEDED libamdhip64.so.7 resolves to it: the stepper runs on torch's HIP
runtime, while the standalone probe binary runs on /opt/rocm's. This script imports torch,
then loads the probe as a shared library and runs it, so its output can be compared line by
line with the standalone binary's.
    python scripts/graph_event_probe_torch.py [iters] [spin_us]
"""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main() -> int:
    import torch

    torch.cuda.init()  # torch's HIP runtime is now the process's
    maps = sorted({ln.split()[-1] for ln in open("/proc/self/maps") if "amdhip64" in ln})
    print('{"amdhip64_mapped": %s, "torch_version_hip": "%s"}' % ([m for m in maps],
                                                                  torch.version.hip), flush=True)
    lib = ctypes.CDLL(os.path.join(ROOT, "gravity-simulator-using-mpi-spark-and-cuda_amd",
                                   "_native", "libgraph_event_probe.so"))
    iters = int(sys.argv[1]) if len(sys.argv) > 1 else 6
    spin = int(sys.argv[2]) if len(sys.argv) > 2 else 20000
    return int(lib.gs_graph_event_probe(iters, spin))


if __name__ == "__main__":
    sys.exit(main())
