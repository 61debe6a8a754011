"""Training engine: Trainer, checkpoints, dry run, optimizers."""

from llmtrain.training.checkpoint import CheckpointManager, CheckpointPayload
from llmtrain.training.trainer import Trainer, TrainResult

__all__ = ["CheckpointManager", "CheckpointPayload", "TrainResult", "Trainer"]
