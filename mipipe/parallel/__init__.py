"""Scale-out pipeline runtime: one process per MI355X, RCCL point-to-point."""
from .engine import PipelineEngine, StepStats, schedule_actions
from .p2p import P2P
from .stage import StagePlan, plan_stages

__all__ = ["PipelineEngine", "StepStats", "schedule_actions", "P2P", "StagePlan", "plan_stages"]
