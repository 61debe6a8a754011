"""Model-adapter registry (``@register_model("gpt")``)."""

from __future__ import annotations

from collections.abc import Callable
from typing import TYPE_CHECKING, TypeVar

from llmtrain.registry.core import Registry, RegistryError

if TYPE_CHECKING:
    from llmtrain.models.base import ModelAdapter

__all__ = ["RegistryError", "available_model_adapters", "get_model_adapter", "register_model"]

A = TypeVar("A")
MODELS: Registry = Registry("Model adapter")


def register_model(name: str) -> Callable[[type[A]], type[A]]:
    return MODELS.register(name)


def get_model_adapter(name: str) -> type[ModelAdapter]:
    return MODELS.get(name)


def available_model_adapters() -> list[str]:
    return MODELS.names()
