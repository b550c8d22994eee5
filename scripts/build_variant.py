"""Build libgravsim_hip.so from a modified copy of csrc into another directory (A/B runs of
code-generation effects; nothing in the tree changes).
    python scripts/build_variant.py --out abv/varA [--patch file:old_text_file:new_text_file]
                                    [--extra "-mllvm -align-loops=64"]
Run the variant with GRAVSIM_NATIVE_DIR=<out> (same Python, same C ABI)."""
import argparse
import os
import shutil
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "csrc"))


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", required=True)
    ap.add_argument("--patch", action="append", default=[],
                    help="rel/path:old.txt:new.txt (replace the text of old.txt by new.txt once)")
    ap.add_argument("--extra", default="", help="extra hipcc flags")
    a = ap.parse_args()
    import build as nb

    tmp = tempfile.mkdtemp(prefix="gravsim_variant_")
    shutil.copytree(os.path.join(ROOT, "csrc"), os.path.join(tmp, "csrc"))
    for p in a.patch:
        rel, old_f, new_f = p.split(":")
        path = os.path.join(tmp, rel)
        src = open(path).read()
        old, new = open(old_f).read(), open(new_f).read()
        assert src.count(old) == 1, f"patch site of {old_f} not found once in {rel}"
        open(path, "w").write(src.replace(old, new))
    os.makedirs(a.out, exist_ok=True)
    srcs = [os.path.join(tmp, os.path.relpath(str(p), ROOT)) for p in nb.HIP_SRC]
    cmd = [nb.hipcc(), *nb.HIP_FLAGS, *a.extra.split(), "-shared",
           f"-I{os.path.join(tmp, 'csrc', 'include')}", *srcs, f"-L{nb.ROCM / 'lib'}", "-lrccl",
           "-o", os.path.join(a.out, "libgravsim_hip.so")]
    subprocess.run(cmd, check=True)
    shutil.copy(nb.CPU_LIB, os.path.join(a.out, "libgravsim_cpu.so"))
    shutil.rmtree(tmp, ignore_errors=True)
    print(f"variant built in {a.out}")
    return 0


if __name__ == "__main__":
    sys.exit(main())
