"""Binary checkpoints and resume (absent from the reference: SURVEY.md §5).

Format (little-endian, rank-agnostic global body order):
    magic   8 B   b"GRAVSIM1"
    header  JSON  (u32 length + UTF-8): n, step, time, dt, dtype, G, cutoff, softening,
                  init, seed, version
    pos     n*3 float64
    vel     n*3 float64
    mass    n   float64
State is always stored in fp64 so an fp32 run resumes exactly (fp32 -> fp64 -> fp32 is exact).
Writes go to a temp file + rename, so a crash never leaves a torn checkpoint.
"""
from __future__ import annotations

import json
import os
import struct
from dataclasses import dataclass

import numpy as np

from ..models.initial_conditions import BodySet

MAGIC = b"GRAVSIM1"


@dataclass
class Checkpoint:
    bodies: BodySet
    step: int
    meta: dict


def save(path: str, bodies: BodySet, step: int, meta: dict) -> str:
    n = bodies.n
    head = dict(meta)
    head.update(n=n, step=int(step), version=1)
    hb = json.dumps(head, sort_keys=True).encode()
    d = os.path.dirname(os.path.abspath(path))
    os.makedirs(d, exist_ok=True)
    tmp = path + ".tmp"
    with open(tmp, "wb") as f:
        f.write(MAGIC)
        f.write(struct.pack("<I", len(hb)))
        f.write(hb)
        f.write(np.ascontiguousarray(bodies.pos, dtype="<f8").tobytes())
        f.write(np.ascontiguousarray(bodies.vel, dtype="<f8").tobytes())
        f.write(np.ascontiguousarray(bodies.mass, dtype="<f8").tobytes())
    os.replace(tmp, path)
    return path


def load(path: str) -> Checkpoint:
    with open(path, "rb") as f:
        if f.read(8) != MAGIC:
            raise ValueError(f"{path}: not a gravsim checkpoint")
        (hl,) = struct.unpack("<I", f.read(4))
        head = json.loads(f.read(hl).decode())
        n = int(head["n"])
        pos = np.frombuffer(f.read(n * 24), dtype="<f8").reshape(n, 3).copy()
        vel = np.frombuffer(f.read(n * 24), dtype="<f8").reshape(n, 3).copy()
        mass = np.frombuffer(f.read(n * 8), dtype="<f8").copy()
        if mass.shape[0] != n:
            raise ValueError(f"{path}: truncated checkpoint")
    return Checkpoint(BodySet(pos, vel, mass), int(head["step"]), head)


def path_for(directory: str, step: int) -> str:
    return os.path.join(directory, f"ckpt_{step:08d}.gsck")


def latest(directory: str) -> str | None:
    if not os.path.isdir(directory):
        return None
    c = sorted(f for f in os.listdir(directory) if f.startswith("ckpt_") and f.endswith(".gsck"))
    return os.path.join(directory, c[-1]) if c else None
