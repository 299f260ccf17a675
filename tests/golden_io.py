"""Loading helpers for the committed golden fixtures (tests/golden/*.npz, *.json).

The fixtures were produced by running the reference (tests/golden/gen_golden.py);
this module only reads data.
"""
from __future__ import annotations

import json
import os

import numpy as np

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
MAP_DIR = os.path.join(REPO, "marl-delivery_amd", "marl_gpu", "maps")


def npz(name):
    return np.load(os.path.join(GOLDEN, name), allow_pickle=False)


def meta(d):
    return json.loads(bytes(d["meta"]).decode())


def load_json(name):
    with open(os.path.join(GOLDEN, name)) as f:
        return json.load(f)


def grid(name):
    rows = []
    with open(os.path.join(MAP_DIR, name)) as f:
        for line in f:
            rows.append([int(x) for x in line.strip().split(" ")])
    return np.asarray(rows, np.uint8)


TRAINER_MOVE_CODES = np.array([4, 1, 2, 0, 3], np.uint8)   # D,L,R,S,U -> S=0,L=1,R=2,U=3,D=4


def decode_trainer(ints):
    """MAPPO/trainer.py:198-205 int -> (move code, op code)."""
    ints = np.asarray(ints).astype(np.int64)
    mv = TRAINER_MOVE_CODES[ints % 5]
    op = ints // 5
    op = np.where(op >= 3, 0, op).astype(np.uint8)
    return mv, op


def trk_rows_from_dict(trk):
    return np.array([[v["id"], 1 if v["status"] == "waiting" else 2, v["start_pos"][0], v["start_pos"][1],
                      v["target_pos"][0], v["target_pos"][1], v["start_time"], v["deadline"]] for v in trk.values()],
                    np.int32).reshape(-1, 8)
