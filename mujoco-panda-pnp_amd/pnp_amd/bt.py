"""Behaviour tree of the pick-and-place demo (reference panda_mujoco_gym/behavior_tree: nodes/pick.py,
nodes/place.py, nodes/home.py, trees/pnp_tree.py) over this engine's skills.

py_trees 2.2.2 is not installed here, so the part of it the reference uses is restated:
``Behaviour.tick`` (initialise when not RUNNING, update, terminate + status on leaving RUNNING),
``Sequence(memory=True)`` (children in order; a child that succeeds hands the same tick to the
next one; restarts from the first child once it has finished) and ``Retry(num_failures)``.  The
node classes keep the reference's phase logic line for line, including its quirks: PickNode
appends its later skills lazily and never re-creates them, PlaceNode rebuilds its skills on every
start, HomeNode moves to ``env.home_pos`` over 30 steps.
"""
from __future__ import annotations

import enum
import types
from typing import Any, Dict, List

from . import skills as _default_skills

# the skill classes the nodes build (a namespace: the batched runner, pnp_amd.batched_bt, passes
# variants whose IK goes through its batched server)
DEFAULT_SKILLS = types.SimpleNamespace(RotateSkill=_default_skills.RotateSkill, MoveIKSkill=_default_skills.MoveIKSkill,
                                       MoveSkill=_default_skills.MoveSkill, GripperSkill=_default_skills.GripperSkill)


class Status(enum.Enum):
    SUCCESS = "SUCCESS"
    FAILURE = "FAILURE"
    RUNNING = "RUNNING"
    INVALID = "INVALID"


class Behaviour:
    """py_trees.behaviour.Behaviour: tick() = [initialise] -> update -> [terminate]."""

    def __init__(self, name: str = ""):
        self.name = name
        self.status = Status.INVALID

    def initialise(self) -> None:
        pass

    def update(self) -> Status:
        return Status.INVALID

    def terminate(self, new_status: Status) -> None:
        pass

    def stop(self, new_status: Status = Status.INVALID) -> None:
        self.terminate(new_status)
        self.status = new_status

    def tick(self) -> Status:
        if self.status != Status.RUNNING:
            self.initialise()
        new_status = self.update()
        if new_status != Status.RUNNING:
            self.stop(new_status)
        self.status = new_status
        return new_status


class Sequence(Behaviour):
    """py_trees.composites.Sequence with memory=True."""

    def __init__(self, name: str = "", children: List[Behaviour] | None = None):
        super().__init__(name)
        self.children: List[Behaviour] = list(children or [])
        self.current = 0

    def add_child(self, child: Behaviour) -> None:
        self.children.append(child)

    def add_children(self, children: List[Behaviour]) -> None:
        self.children.extend(children)

    def tick(self) -> Status:
        if self.status != Status.RUNNING:
            self.current = 0
            for c in self.children:
                if c.status != Status.INVALID:
                    c.stop(Status.INVALID)
        while self.current < len(self.children):
            st = self.children[self.current].tick()
            if st != Status.SUCCESS:
                self.status = st
                return st
            self.current += 1
        self.stop(Status.SUCCESS)
        return Status.SUCCESS


class Retry(Behaviour):
    """py_trees.decorators.Retry: re-run the child after a failure, up to num_failures times."""

    def __init__(self, name: str, child: Behaviour, num_failures: int):
        super().__init__(name)
        self.child, self.num_failures, self.failures = child, num_failures, 0

    def initialise(self) -> None:
        self.failures = 0

    def update(self) -> Status:
        st = self.child.tick()
        if st == Status.FAILURE:
            self.failures += 1
            if self.failures < self.num_failures:
                self.child.stop(Status.INVALID)
                return Status.RUNNING
            return Status.FAILURE
        return st

    def stop(self, new_status: Status = Status.INVALID) -> None:
        """py_trees.decorators.Decorator.stop: an INVALID stop (a parent resetting) stops the
        child too, and a child still RUNNING is stopped whatever the decorator's own status."""
        self.terminate(new_status)
        if new_status == Status.INVALID:
            self.child.stop(new_status)
        if self.child.status == Status.RUNNING:
            self.child.stop(Status.INVALID)
        self.status = new_status


class BehaviourTree:
    def __init__(self, root: Behaviour):
        self.root = root
        self.count = 0

    def tick(self) -> Status:
        self.count += 1
        return self.root.tick()


# ----------------------------------------------------------------------------- nodes
class PickNode(Behaviour):
    """nodes/pick.py: Rotate -> MoveIK approach_wpt1 -> MoveIK obj_pos -> Grasp -> MoveIK approach_wpt2."""

    def __init__(self, env: Any, meta: Dict[str, Any], name: str | None = None, skills=None):
        super().__init__(name or f"Pick-{meta.get('id', 'obj')}")
        self.env, self.meta = env, meta
        self.sk = skills or DEFAULT_SKILLS
        self.skills: List[Any] = [self.sk.RotateSkill(env, meta["delta_q"])]
        self.phase = 0
        self.curr = None

    def initialise(self) -> None:
        self.phase = 0
        for sk in self.skills:
            sk.reset()
        self.curr = self.skills[0]

    def update(self) -> Status:
        self.curr.step()
        if getattr(self.curr, "done", False):
            self.phase += 1
            if self.phase == 1:
                self.skills.append(self.sk.MoveIKSkill(self.env, self.meta["approach_wpt1"]))
            elif self.phase == 2:
                self.skills.append(self.sk.MoveIKSkill(self.env, self.meta["obj_pos"]))
            elif self.phase == 3:
                self.skills.append(self.sk.GripperSkill.close(self.env))
            elif self.phase == 4:
                self.skills.append(self.sk.MoveIKSkill(self.env, self.meta["approach_wpt2"]))
            if self.phase >= len(self.skills):
                return Status.SUCCESS
            self.curr = self.skills[self.phase]
            self.curr.reset()
        return Status.RUNNING

    @property
    def done(self) -> bool:
        return self.status == Status.SUCCESS


class PlaceNode(Behaviour):
    """nodes/place.py: MoveIK approach_wpt1 -> MoveIK home_wpt -> Rotate back -> MoveIK approach_wpt2 -> open."""

    def __init__(self, env: Any, meta: Dict[str, Any], name: str = "Place", skills=None):
        super().__init__(name)
        self.env, self.meta = env, meta
        self.sk = skills or DEFAULT_SKILLS
        self.skills: List[Any] = []
        self.phase = 0
        self.curr = None

    def initialise(self) -> None:
        self.skills.clear()
        self.phase = 0
        self.curr = self._build_skill(self.phase)
        self.curr.reset()

    def update(self) -> Status:
        self.curr.step()
        if getattr(self.curr, "done", False):
            self.phase += 1
            if self.phase >= 5:
                return Status.SUCCESS
            self.curr = self._build_skill(self.phase)
            self.curr.reset()
            self.skills.append(self.curr)
        return Status.RUNNING

    def _build_skill(self, phase: int):
        if phase == 0:
            return self.sk.MoveIKSkill(self.env, self.meta["approach_wpt1"])
        if phase == 1:
            return self.sk.MoveIKSkill(self.env, self.meta["home_wpt"])
        if phase == 2:
            return self.sk.RotateSkill(self.env, self.meta["rotate_back_quat"])
        if phase == 3:
            return self.sk.MoveIKSkill(self.env, self.meta["approach_wpt2"])
        if phase == 4:
            return self.sk.GripperSkill.open(self.env)
        raise ValueError(f"[PlaceNode] Invalid phase {phase}")

    def terminate(self, new_status: Status) -> None:
        if new_status == Status.INVALID:
            for sk in self.skills[self.phase:]:
                sk.reset()

    @property
    def done(self) -> bool:
        return self.status == Status.SUCCESS


class HomeNode(Behaviour):
    """nodes/home.py: MoveSkill to env.home_pos over 30 steps."""

    def __init__(self, env: Any, name: str = "Home", skills=None):
        super().__init__(name)
        self.env = env
        self.sk = skills or DEFAULT_SKILLS
        self.skill = None

    def initialise(self) -> None:
        home_pos = getattr(self.env, "home_pos", None)
        if home_pos is None:
            home_pos = self.env.get_ee_position()
        self.skill = self.sk.MoveSkill(self.env, target_pos=home_pos, steps=30)
        self.skill.reset()

    def update(self) -> Status:
        self.skill.step()
        return Status.SUCCESS if self.skill.done else Status.RUNNING

    def terminate(self, new_status: Status) -> None:
        if new_status == Status.INVALID and self.skill is not None:
            self.skill.reset()

    @property
    def done(self) -> bool:
        return self.status == Status.SUCCESS


def build_pnp_tree(env: Any, tasks: List[Dict[str, Any]], retry_pick: int = 3, skills=None) -> BehaviourTree:
    """trees/pnp_tree.py: root Sequence(memory) of per-object Sequence(Pick [Retry], Place, Home).
    ``skills``: the skill classes the nodes build (default: pnp_amd.skills)."""
    root = Sequence(name="PnP-Root")
    for i, task in enumerate(tasks):
        pick: Behaviour = PickNode(env, meta=task["obj_meta"], name=f"Pick-{i}", skills=skills)
        if retry_pick > 1:
            pick = Retry(name=f"RetryPick-{i}", child=pick, num_failures=retry_pick)
        place = PlaceNode(env, meta=task["place_meta"], name=f"Place-{i}", skills=skills)
        home = HomeNode(env, name=f"Home-{i}", skills=skills)
        sub = Sequence(name=f"PnP-Task-{i}")
        sub.add_children([pick, place, home])
        root.add_child(sub)
    return BehaviourTree(root)
