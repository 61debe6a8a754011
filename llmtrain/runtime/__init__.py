"""Runtime policy (device / precision / seeding) and flat parameter storage."""

from llmtrain.runtime.device import RuntimePolicy, resolve_policy, seed_everything
from llmtrain.runtime.flat import FlatParamStore

__all__ = ["FlatParamStore", "RuntimePolicy", "resolve_policy", "seed_everything"]
