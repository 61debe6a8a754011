"""Configuration schema and loader."""

from llmtrain.config.loader import ConfigLoadError, load_and_validate_config
from llmtrain.config.schemas import (
    DataConfig,
    DDPConfig,
    LoggingConfig,
    MLflowConfig,
    ModelConfig,
    OutputConfig,
    RunConfig,
    RunSectionConfig,
    TrainerConfig,
)

__all__ = [
    "ConfigLoadError",
    "DataConfig",
    "DDPConfig",
    "LoggingConfig",
    "MLflowConfig",
    "ModelConfig",
    "OutputConfig",
    "RunConfig",
    "RunSectionConfig",
    "TrainerConfig",
    "load_and_validate_config",
]
