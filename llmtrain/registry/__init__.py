"""Plugin registries. ``initialize_registries()`` imports the built-in plugins so their
decorators run (reference ``registry/__init__.py:7-20``)."""

from __future__ import annotations

from importlib import import_module

from llmtrain.registry.core import Registry, RegistryError

MODEL_REGISTRY_MODULES: tuple[str, ...] = (
    "llmtrain.models.dummy_gpt",
    "llmtrain.models.gpt",
)
DATA_REGISTRY_MODULES: tuple[str, ...] = (
    "llmtrain.data.dummy_text",
    "llmtrain.data.hf_text",
    "llmtrain.data.synthetic_tokens",
)

__all__ = ["Registry", "RegistryError", "initialize_registries"]


def initialize_registries() -> None:
    for module in MODEL_REGISTRY_MODULES + DATA_REGISTRY_MODULES:
        import_module(module)
