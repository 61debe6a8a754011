"""Compatibility import path of the reference (``llmtrain.distributed``)."""

from llmtrain.parallel.dist import DDPState, setup_ddp, teardown_ddp

__all__ = ["DDPState", "setup_ddp", "teardown_ddp"]
