"""A/B of the sym force launch's first wave (workgroups that take one unit each before the
dynamic fetch takes up to dyn_cap; the default is occupancy x CUs) on one GPU, alternating
values within each round on one engine per size.

    python scripts/first_wave_ab.py --n 65536,1048576 --waves 512,256,1024,1 --rounds 3
    python scripts/first_wave_ab.py --n 65536 --waves 512 --caps 3,4,6,8   (the dynamic cap)
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
    ap.add_argument("--caps", default="", help="dynamic-fetch caps to alternate (default: as is)")
    ap.add_argument("--persist", default="", help="persistent-workgroup modes to alternate (1,0)")
    a = ap.parse_args()
    import gravsim  # noqa: F401
    from gravsim.config import SimConfig
    from gravsim.runtime.engines import HipEngine

    for n in [int(x) for x in a.n.split(",")]:
        # about 0.3 s per measurement (0.7 ms per step at 65K, quadratic in n)
        steps = max(6, min(400, int(0.3 / (0.7e-3 * (n / 65536) ** 2))))
        e = HipEngine(SimConfig(n=n, dtype="fp32", device="gpu"), 0, 1)
        e.init_ics("solar+random", 1)
        caps = [int(x) for x in a.caps.split(",")] if a.caps else [e.dyn_cap]
        pers = [int(x) for x in a.persist.split(",")] if a.persist else [-1]
        for rnd in range(a.rounds):
            for w in [int(x) for x in a.waves.split(",")]:
                for cap, pe in [(c, p) for c in caps for p in pers]:
                    e.set_tuning(first_wave=w, persist=pe)
                    e.set_schedule(1, cap)
                    e.step(4)
                    e.sync()
                    t0 = time.perf_counter()
                    e.step(steps)
                    e.sync()
                    ms = 1e3 * (time.perf_counter() - t0) / steps
                    print(json.dumps(dict(n=n, round=rnd, first_wave=w, dyn_cap=cap, persist=pe,
                                          steps=steps, ms_per_step=ms)), flush=True)
        e.close()
    return 0


if __name__ == "__main__":
    sys.exit(main())
