"""Hash of the state after a few sym steps (one GPU): compares native builds bit for bit.
    GRAVSIM_NATIVE_DIR=<dir> python scripts/state_hash.py [--n N] [--steps K] [--dtype fp32]
    python scripts/state_hash.py --cases 65536:fp32:auto:1,1048576:fp32:auto:1,...
A case is n:dtype:cutoff_mode:P; P > 1 runs P virtual ranks on the one GPU (the multi-rank
sym schedule with the exchanges as device copies). Prints one JSON line per case
{"native": dir, "n": N, "steps": K, "sha": <sha256 of pos+vel>}."""
import argparse
import hashlib
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def one(n: int, dtype: str, cutoff: str, P: int, steps: int) -> dict:
    import gravsim  # noqa: F401
    from gravsim.config import SimConfig
    from gravsim.runtime.engines import HipEngine, VirtualGroup

    cfg = SimConfig(n=n, dtype=dtype, device="gpu", mode="sym", cutoff_mode=cutoff).validate()
    eng = VirtualGroup(cfg, P) if P > 1 else HipEngine(cfg, device=0)
    try:
        eng.init_ics("solar+random", cfg.seed)
        eng.step(steps)
        eng.sync()
        b = eng.state()
        h = hashlib.sha256(b.pos.tobytes() + b.vel.tobytes()).hexdigest()[:16]
    finally:
        eng.close()
    return {"native": os.environ.get("GRAVSIM_NATIVE_DIR", "in-tree"), "n": n, "steps": steps,
            "dtype": dtype, "cutoff": cutoff, "P": P, "sha": h}


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=65536)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--dtype", default="fp32")
    ap.add_argument("--cutoff-mode", default="auto")
    ap.add_argument("--cases", default="", help="n:dtype:cutoff:P,... (overrides --n/--dtype)")
    a = ap.parse_args()
    cases = [(a.n, a.dtype, a.cutoff_mode, 1)]
    if a.cases:
        cases = []
        for c in a.cases.split(","):
            n, dt, cut, P = c.split(":")
            cases.append((int(n), dt, cut, int(P)))
    for n, dt, cut, P in cases:
        print(json.dumps(one(n, dt, cut, P, a.steps)), flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
