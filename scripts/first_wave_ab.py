"""A/B of the sym force launch's first wave (workgroups that take one unit each before the
dynamic fetch takes up to dyn_cap; the default is occupancy x CUs) on one GPU, alternating
values within each round on one engine per size.

    python scripts/first_wave_ab.py --n 65536,1048576 --waves 512,256,1024,1 --rounds 3
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", default="65536,1048576")
    ap.add_argument("--waves", default="512,256,1024,1")
    ap.add_argument("--rounds", type=int, default=3)
    a = ap.parse_args()
    import gravsim  # noqa: F401
    from gravsim.config import SimConfig
    from gravsim.runtime.engines import HipEngine

    for n in [int(x) for x in a.n.split(",")]:
        # about 0.3 s per measurement (0.7 ms per step at 65K, quadratic in n)
        steps = max(6, min(400, int(0.3 / (0.7e-3 * (n / 65536) ** 2))))
        e = HipEngine(SimConfig(n=n, dtype="fp32", device="gpu"), 0, 1)
        e.init_ics("solar+random", 1)
        for rnd in range(a.rounds):
            for w in [int(x) for x in a.waves.split(",")]:
                e.set_tuning(first_wave=w)
                e.step(4)
                e.sync()
                t0 = time.perf_counter()
                e.step(steps)
                e.sync()
                ms = 1e3 * (time.perf_counter() - t0) / steps
                print(json.dumps(dict(n=n, round=rnd, first_wave=w, steps=steps, ms_per_step=ms)),
                      flush=True)
        e.close()
    return 0


if __name__ == "__main__":
    sys.exit(main())
