"""Loading helpers for the committed golden fixtures (tests/golden/*.npz).

The fixtures were produced by tests/golden/make_golden.py from the reference
updater itself; they are data only (inputs and expected outputs).
"""
from __future__ import annotations

import glob
import json
import os

import numpy as np

GOLDEN_DIR = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")

STATE_KEYS = ["p_x", "p_y", "p_depth", "p_health", "st_x", "st_y", "tick", "status", "episode",
              "ret_sum", "ep_count", "counters", "npc_pos", "npc_health", "npc_alive"]


def case_names():
    """Trajectory fixtures (every npz but the known-answer scenario table)."""
    return sorted(os.path.splitext(os.path.basename(p))[0]
                  for p in glob.glob(os.path.join(GOLDEN_DIR, "*.npz"))
                  if not os.path.basename(p).startswith("kat_"))


class Fixture:
    def __init__(self, name: str):
        self.name = name
        z = np.load(os.path.join(GOLDEN_DIR, name + ".npz"), allow_pickle=False)
        self.z = {k: z[k] for k in z.files}
        self.cfg = json.loads(bytes(self.z["cfg_json"]).decode())
        self.seed = int(self.z["seed"][0])
        self.game_offset = int(self.z["game_offset"][0])
        self.actions = self.z["actions"]            # [T, G, 2] int8
        self.T, self.G = self.actions.shape[:2]
        self.K = int(self.cfg["n_npcs"])
        self.policy = tuple(self.cfg["policy"])
        # stock-seed fixture (cfg.rng = MT19937): bots and shuffles share each
        # game's random stream, so a step must follow that tick's policy draws
        self.stock = int(self.cfg.get("rng", 0)) == 1
        # explicit-grid cases: the dungeon bank ([L, W, H] Tile codes), else None
        self.layouts = self.z.get("layouts")
        wl = self.z["world_len"]
        self._world_off = np.concatenate([[0], np.cumsum(wl.ravel())])
        el = self.z["event_len"]
        self._ev_off = np.concatenate([[0], np.cumsum(el.ravel())])
        nl = self.z["entity_len"]
        self._ent_off = np.concatenate([[0], np.cumsum(nl.ravel())])

    def serialized(self, t: int, g: int) -> bytes:
        """serializer.serialize(GameState) of game g after t steps (t must be in
        ser_ticks)."""
        j = list(self.z["ser_ticks"]).index(t)
        lens = self.z["ser_len"]
        start = int(lens[:j].sum() + lens[j, :g].sum())
        return bytes(self.z["ser_bytes"][start:start + int(lens[j, g])])

    def state(self, t: int) -> dict:
        """Engine-layout state after t steps (t = 0: after the initial reset)."""
        out = {k: self.z[k][t] for k in STATE_KEYS}
        if "p_layout" in self.z:
            out["p_layout"] = self.z["p_layout"][t]
        return out

    def world(self, t: int, g: int):
        i = t * self.G + g
        rows = self.z["world"][self._world_off[i]:self._world_off[i + 1]]
        return [tuple(int(v) for v in r) for r in rows]

    def events(self, t: int, g: int):
        """Update events of step t (0-based) of game g."""
        i = t * self.G + g
        rows = self.z["events"][self._ev_off[i]:self._ev_off[i + 1]]
        return [tuple(int(v) for v in r) for r in rows]

    def entities(self, t: int, g: int):
        i = t * self.G + g
        rows = self.z["entities"][self._ent_off[i]:self._ent_off[i + 1]]
        return [tuple(int(v) for v in r) for r in rows]


def compare_state(got: dict, want: dict, K: int, where: str = ""):
    """Asserts bit-exact equality of every state field (NPC slots only if K;
    the bank layout of each player's depth when both sides carry it)."""
    keys = STATE_KEYS + [k for k in ("p_layout", "sep_start", "p_rpg", "item_mask", "item_pos")
                         if k in got and k in want]
    for k in keys:
        if k.startswith("npc") and K == 0:
            continue
        g = np.asarray(got[k])
        w = np.asarray(want[k])
        if k in ("npc_pos", "npc_health", "item_pos"):
            # dead NPC slots / taken items are unspecified: compare live slots only
            from optimax_rogue_amd.enums import npc_alive_bits
            mask = npc_alive_bits(want["item_mask"][0] if k == "item_pos" else want["npc_alive"], K)
            g = np.where(mask, g, 0)
            w = np.where(mask, w, 0)
        if g.shape != w.shape or not np.array_equal(g.astype(np.int64), w.astype(np.int64)):
            bad = np.argwhere(g.astype(np.int64) != w.astype(np.int64)) if g.shape == w.shape else None
            raise AssertionError(f"{where}: field {k} differs; first mismatches {bad[:5] if bad is not None else 'shape'}"
                                 f"\n got={g.ravel()[:16]}\nwant={w.ravel()[:16]}")


class Kat:
    """tests/golden/kat_scenarios.npz: SURVEY.md s4's semantics probes (swap,
    block, same target, chase, wall, descend, NPC kill ...) as hand-built
    one-tick states stepped by the reference updater (make_golden.py
    make_scenarios)."""

    def __init__(self):
        self.z = np.load(os.path.join(GOLDEN_DIR, "kat_scenarios.npz"))
        self.cfg = json.loads(bytes(self.z["cfg_json"]).decode())
        self.names = [str(n) for n in self.z["names"]]
        self._ev = np.concatenate([[0], np.cumsum(self.z["ev_len"])])
        self._en = np.concatenate([[0], np.cumsum(self.z["ent_len"])])

    def case(self, i):
        z = self.z
        ents = [tuple(int(v) for v in e) for e in z["init"][i] if e[0] >= 0]
        events = [tuple(int(v) for v in r) for r in z["events"][self._ev[i]:self._ev[i + 1]]]
        final = {k[6:]: z[k][i] for k in z.files if k.startswith("final_")}
        out_ents = [tuple(int(v) for v in r) for r in z["ents"][self._en[i]:self._en[i + 1]]]
        return dict(name=self.names[i], ents=ents, moves=[int(v) for v in z["moves"][i]],
                    seed=int(z["seeds"][i]), events=events, final=final, entities=out_ents)
