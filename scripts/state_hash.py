"""Hash of the state after a few sym steps (one GPU): compares native builds bit for bit.
    GRAVSIM_NATIVE_DIR=<dir> python scripts/state_hash.py [--n N] [--steps K] [--dtype fp32]
Prints one JSON line {"native": dir, "n": N, "steps": K, "sha": <sha256 of pos+vel>}."""
import argparse
import hashlib
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=65536)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--dtype", default="fp32")
    ap.add_argument("--cutoff-mode", default="auto")
    a = ap.parse_args()
    import gravsim  # noqa: F401
    from gravsim.config import SimConfig
    from gravsim.runtime.engines import HipEngine

    cfg = SimConfig(n=a.n, dtype=a.dtype, device="gpu", mode="sym",
                    cutoff_mode=a.cutoff_mode).validate()
    eng = HipEngine(cfg, device=0)
    try:
        eng.init_ics("solar+random", cfg.seed)
        eng.step(a.steps)
        eng.sync()
        b = eng.state()
        h = hashlib.sha256(b.pos.tobytes() + b.vel.tobytes()).hexdigest()[:16]
    finally:
        eng.close()
    print(json.dumps({"native": os.environ.get("GRAVSIM_NATIVE_DIR", "in-tree"), "n": a.n,
                      "steps": a.steps, "dtype": a.dtype, "cutoff": a.cutoff_mode, "sha": h}))
    return 0


if __name__ == "__main__":
    sys.exit(main())
