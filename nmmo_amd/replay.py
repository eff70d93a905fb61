"""Replay files: nmmo's FileReplayHelper over the single-env facade.

The reference records a replay by attaching a helper to the env's realm, resetting it, stepping
the env, and saving one compressed file (train_helper.py:132-134, :171, :229-235):

    replay_helper = FileReplayHelper()
    nmmo_env.realm.record_replay(replay_helper)
    replay_helper.reset()
    ... env steps ...
    replay_helper.save(replay_file, compress=True)     # -> replay_file + ".replay.lzma"

File format **[recalled: nmmo 2.1 nmmo/render/replay_helper.py; not in the reference tree,
unpinned]**: `json.dumps({"map": ..., "packets": [...]})` encoded UTF-8 and, with
compress=True, `lzma.compress(..., format=lzma.FORMAT_ALONE)` under `<prefix>.replay.lzma`
(`<prefix>.replay.json` uncompressed). "map" is the material grid at reset; each packet is one
tick of the realm: every entity in the realm keyed by id under "player" / "npc" with its
position, level, resources, skills and combat status (the Entity columns of SPEC §7), the
tiles whose material changed since the previous packet, and the tick's event-log rows.
"""

from __future__ import annotations

import json
import lzma

import numpy as np

from . import abi

SKILLS = ("melee", "range", "mage", "fishing", "herbalism", "prospecting", "carving", "alchemy")


def _entity_packet(ent: dict, s: int) -> dict:
    g = {k: int(v[s]) for k, v in ent.items()}
    level = max(g["melee_level"], g["range_level"], g["mage_level"])
    return {
        "base": {"r": g["row"], "c": g["col"], "level": level, "item_level": g["item_level"],
                 "population": 0 if g["id"] > 0 else -g["npc_type"], "name": f"{'Player' if g['id'] > 0 else 'NPC'}_{abs(g['id'])}",
                 "gold": g["gold"]},
        "resource": {k: {"val": g[k], "max": 100} for k in ("health", "food", "water")},
        "skills": {k: {"level": g[f"{k}_level"], "exp": g[f"{k}_exp"]} for k in SKILLS},
        "status": {"freeze": g["freeze"]},
        "history": {"damage": g["damage"], "time_alive": g["time_alive"],
                    "attacker_id": g["attacker_id"], "latest_combat_tick": g["latest_combat_tick"]},
        "alive": bool(g["alive"]) and g["health"] > 0,
    }


def packet(state: dict, events: np.ndarray, prev_mat: np.ndarray | None) -> dict:
    """One tick of the realm from NmmoEnv.state() and the tick's event rows."""
    ent = state["entities"]
    players, npcs = {}, {}
    for s in range(len(ent["id"])):
        eid = int(ent["id"][s])
        if eid == 0 or not ent["alive"][s]:
            continue
        (players if eid > 0 else npcs)[eid] = _entity_packet(ent, s)
    mat = state["material"]
    changed = [] if prev_mat is None else [[int(r), int(c), int(mat[r, c])]
                                          for r, c in zip(*np.nonzero(mat != prev_mat))]
    tick = state["tick"]
    ev = events[events[:, abi.ATTR_TO_COL["tick"]] == tick] if len(events) else events
    return {"tick": tick, "player": players, "npc": npcs, "resource": changed,
            "event": ev.astype(int).tolist()}


class FileReplayHelper:
    """nmmo.render.replay_helper.FileReplayHelper shape: reset(), update(), save(prefix, compress)."""

    def __init__(self):
        self._env = None
        self.map = None
        self.packets = []
        self._prev_mat = None

    def set_env(self, env):  # realm.record_replay(helper) -> env.record_replay(helper)
        self._env = env

    def reset(self):
        self.packets = []
        self.map = None
        self._prev_mat = None
        self.update()

    def update(self):
        if self._env is None:
            return
        st = self._env.state()
        if self.map is None:
            self.map = st["material"].astype(int).tolist()
        self.packets.append(packet(st, self._env.engine.events(0), self._prev_mat))
        self._prev_mat = st["material"].copy()

    def save(self, filename_prefix: str, compress: bool = True) -> str:
        data = json.dumps({"map": self.map, "packets": self.packets}).encode("utf8")
        if compress:
            path = f"{filename_prefix}.replay.lzma"
            data = lzma.compress(data, format=lzma.FORMAT_ALONE)
        else:
            path = f"{filename_prefix}.replay.json"
        with open(path, "wb") as f:
            f.write(data)
        return path


def load_replay(path: str) -> dict:
    """Inverse of FileReplayHelper.save (either suffix)."""
    raw = open(path, "rb").read()
    if path.endswith(".lzma"):
        raw = lzma.decompress(raw, format=lzma.FORMAT_ALONE)
    return json.loads(raw.decode("utf8"))
