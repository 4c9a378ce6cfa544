"""Scale-out pipeline runtime: one process per MI355X, RCCL point-to-point,
optional data-parallel replicas of the pipeline."""
from .data_parallel import DataParallelGrads, make_pp_dp_groups
from .engine import PipelineEngine, StepStats, schedule_actions
from .p2p import P2P
from .stage import StagePlan, plan_stages

__all__ = ["PipelineEngine", "StepStats", "schedule_actions", "P2P", "StagePlan", "plan_stages",
           "DataParallelGrads", "make_pp_dp_groups"]
