"""Experiment tracking backends."""

from llmtrain.tracking.base import NullTracker, Tracker
from llmtrain.tracking.mlflow import MLflowTracker

__all__ = ["MLflowTracker", "NullTracker", "Tracker"]
