"""Reference-schema update events (optimax_rogue/logic/updates.py) built from
the engine's event records (orx_step_events, include/orx.h ORX_EV_*).

Same class roles and attribute names as the reference:
  EntityCombatUpdate(order, attacker_iden, defender_iden, og_damage, tags,
                     attack_prevals, defend_prevals)          updates.py:71-139
  EntityDeathUpdate(order, entity_iden)                       updates.py:167-184
  EntityPositionUpdate(order, entity_iden, depth, old_depth, posx, posy)
                                                              updates.py:186-220
  DungeonCreatedUpdate(order, depth, dungeon)                 updates.py:308-335
with ``apply(game_state)`` (client-side replication, as optimax_rogue_bots/main.py
does with UpdatePackets) and ``relevant_for(game_state, depth)`` (the server's
per-depth broadcast filter, networking/server.py:171-222), both working on any
object with the GameState surface (compat.GameStateView included), and
``to_prims()`` in the reference's primitive format.
"""
from __future__ import annotations

from typing import List, Optional

from .enums import EV_COMBAT, EV_DEATH, EV_DUNGEON, EV_HEALTH, EV_POSITION, CombatFlag


class GameStateUpdate:
    def __init__(self, order: int):
        self.order = order


class EntityCombatUpdate(GameStateUpdate):
    def __init__(self, order, attacker_iden, defender_iden, og_damage, tags, attack_prevals=(),
                 defend_prevals=()):
        super().__init__(order)
        self.attacker_iden, self.defender_iden = attacker_iden, defender_iden
        self.og_damage = og_damage
        self.tags = set(tags)
        self.attack_prevals, self.defend_prevals = tuple(attack_prevals), tuple(defend_prevals)

    def to_prims(self):
        return {"order": self.order, "attacker_iden": self.attacker_iden,
                "defender_iden": self.defender_iden, "og_damage": self.og_damage,
                "tags": tuple(int(t) for t in self.tags), "attack_prevals": (),
                "defend_prevals": ()}

    def apply(self, game_state) -> None:
        # no Modifier subclass exists, so the hooks are empty (updates.py:117-133)
        if self.og_damage > 0:
            game_state.iden_lookup[self.defender_iden].health -= self.og_damage

    def relevant_for(self, game_state, depth: int) -> bool:
        return (game_state.iden_lookup[self.attacker_iden].depth == depth
                or game_state.iden_lookup[self.defender_iden].depth == depth)


class EntityDeathUpdate(GameStateUpdate):
    def __init__(self, order, entity_iden):
        super().__init__(order)
        self.entity_iden = entity_iden

    def to_prims(self):
        return {"order": self.order, "entity_iden": self.entity_iden}

    def apply(self, game_state) -> None:
        game_state.remove_entity(game_state.iden_lookup[self.entity_iden])

    def relevant_for(self, game_state, depth: int) -> bool:
        return game_state.iden_lookup[self.entity_iden].depth == depth


class EntityPositionUpdate(GameStateUpdate):
    def __init__(self, order, entity_iden, depth, old_depth, posx, posy):
        super().__init__(order)
        self.entity_iden, self.depth, self.old_depth = entity_iden, depth, old_depth
        self.posx, self.posy = posx, posy

    @property
    def depth_changed(self):
        return self.depth != self.old_depth

    def to_prims(self):
        return {"order": self.order, "entity_iden": self.entity_iden, "depth": self.depth,
                "old_depth": self.old_depth, "posx": self.posx, "posy": self.posy}

    def apply(self, game_state) -> None:
        game_state.move_entity(game_state.iden_lookup[self.entity_iden], self.depth, self.posx,
                               self.posy)

    def relevant_for(self, game_state, depth: int) -> bool:
        return depth == self.old_depth


class DungeonCreatedUpdate(GameStateUpdate):
    def __init__(self, order, depth, dungeon):
        super().__init__(order)
        self.depth, self.dungeon = depth, dungeon

    def apply(self, game_state) -> None:
        game_state.world.set_at_depth(self.depth, self.dungeon)

    def relevant_for(self, game_state, depth: int) -> bool:
        return depth == self.depth


class EntityHealthUpdate(GameStateUpdate):
    """Health change outside combat (updates.py:222-253); emitted only by the
    EXT_SEPARATION_DAMAGE build extension (source = the entity itself)."""

    def __init__(self, order, entity_iden, source_iden, amount, tags):
        super().__init__(order)
        self.entity_iden, self.source_iden, self.amount = entity_iden, source_iden, amount
        self.tags = frozenset(tags)

    def to_prims(self):
        return {'order': self.order, 'entity_iden': self.entity_iden,
                'source_iden': self.source_iden, 'amount': self.amount,
                'tags': tuple(self.tags)}

    def apply(self, game_state) -> None:
        game_state.iden_lookup[self.entity_iden].health += self.amount

    def relevant_for(self, game_state, depth: int) -> bool:
        return depth in (game_state.iden_lookup[self.entity_iden].depth,
                         game_state.iden_lookup[self.source_iden].depth)


def from_events(rows, order_start: int, og_damage: int, pre_depth: dict,
                dungeon_for=None, npc_og_damage: Optional[int] = None) -> List[GameStateUpdate]:
    """Update objects for one game's event records [(type, iden, a, b), ...].

    ``order`` continues the Updater's running counter (updater.py:71-74);
    ``og_damage`` = attacker damage - armor (updater.py:313); ``pre_depth``
    maps entity iden -> depth before the tick (EntityPositionUpdate.old_depth;
    an entity moves at most once per tick); ``dungeon_for(depth)`` supplies
    DungeonCreatedUpdate.dungeon (the engine regenerates it from its key);
    ``npc_og_damage`` = an NPC attacker's damage - armor (moving NPCs, whose
    attacks the enemy AI makes; default ``og_damage``)."""
    out: List[GameStateUpdate] = []
    order = order_start
    for typ, iden, a, b in rows:
        if typ == EV_COMBAT:
            og = og_damage if iden <= 2 or npc_og_damage is None else npc_og_damage
            out.append(EntityCombatUpdate(order, iden, a, og, {CombatFlag(b)}))
        elif typ == EV_DEATH:
            out.append(EntityDeathUpdate(order, iden))
        elif typ == EV_POSITION:
            out.append(EntityPositionUpdate(order, iden, a, pre_depth[iden], b & 0xFFFF, b >> 16))
        elif typ == EV_DUNGEON:
            out.append(DungeonCreatedUpdate(order, a, dungeon_for(a) if dungeon_for else None))
        elif typ == EV_HEALTH:
            out.append(EntityHealthUpdate(order, iden, iden, a, {"separation"}))
        else:
            raise ValueError(f"unknown event type {typ}")
        order += 1
    return out
