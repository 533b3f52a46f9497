"""Scripted skills (reference panda_mujoco_gym/skills): same classes, constructor arguments and
tick semantics, driving the device engine through the facade's MuJoCo-binding surface."""
from ..ik_solver import IKResult, JacobianIKController
from .base import Skill
from .gripper import GripperSkill
from .move import MoveIKSkill, MoveSkill, plan_ik_waypoints
from .rotate import RotateSkill

__all__ = ["Skill", "MoveSkill", "MoveIKSkill", "RotateSkill", "GripperSkill", "JacobianIKController", "IKResult",
           "plan_ik_waypoints"]
