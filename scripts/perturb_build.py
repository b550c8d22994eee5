"""Build a deliberately broken copy of libgravsim_hip.so to prove the accuracy gates bite.
    python scripts/perturb_build.py [--out abv/perturbed] [--what carrier]
The copy's sym tile moves one carrier component by the wrong DPP offset (row_ror:2 instead of
row_ror:1 for the x carrier of j-slot 0): the j-side sums of those bodies land on the wrong
lanes. smoke() and tests/test_gpu_scale.py::test_sym_1m_step_path_accel_sampled must FAIL on
it (GRAVSIM_NATIVE_DIR=<out>); scripts/gpu.sh task `perturb` runs both and expects failures.
Built on the CPU host (hipcc cross-compiles gfx950), nothing in the tree changes."""
import argparse
import os
import shutil
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "csrc"))

PERTURB = {
    "carrier": ("    c.cx[0] = row_from<1>(c.cx[0]) - tx.x;",
                "    c.cx[0] = row_from<2>(c.cx[0]) - tx.x;"),
    # the fp64 tile's x carrier (tests/test_gpu_scale.py::test_sym_fp64_512k_bands_accel_sampled
    # and bench.py --dtype fp64's sampled gate must fail on it)
    "carrier64": ("    c.cx[0] = row_from<1>(c.cx[0]) - tx;",
                  "    c.cx[0] = row_from<2>(c.cx[0]) - tx;"),
}


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default=os.path.join(ROOT, "abv", "perturbed"))
    ap.add_argument("--what", default="carrier", choices=sorted(PERTURB))
    a = ap.parse_args()
    import build as nb  # csrc/build.py: the production flags and sources

    tmp = tempfile.mkdtemp(prefix="gravsim_perturb_")
    shutil.copytree(os.path.join(ROOT, "csrc"), os.path.join(tmp, "csrc"))
    hdr = os.path.join(tmp, "csrc", "include", "gs_sym_tile.h")
    old, new = PERTURB[a.what]
    src = open(hdr).read()
    assert src.count(old) == 1, "perturbation site not found"
    open(hdr, "w").write(src.replace(old, new))
    os.makedirs(a.out, exist_ok=True)
    srcs = [os.path.join(tmp, os.path.relpath(str(p), ROOT)) for p in nb.HIP_SRC]
    cmd = [nb.hipcc(), *nb.HIP_FLAGS, "-shared", f"-I{os.path.join(tmp, 'csrc', 'include')}",
           *srcs, f"-L{nb.ROCM / 'lib'}", "-lrccl", "-o", os.path.join(a.out, "libgravsim_hip.so")]
    subprocess.run(cmd, check=True)
    shutil.copy(nb.CPU_LIB, os.path.join(a.out, "libgravsim_cpu.so"))
    shutil.rmtree(tmp, ignore_errors=True)
    print(f"perturbed ({a.what}) build in {a.out}")
    return 0


if __name__ == "__main__":
    sys.exit(main())
