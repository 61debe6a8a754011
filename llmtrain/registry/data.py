"""Data-module registry (``@register_data_module("dummy_text")``)."""

from __future__ import annotations

from collections.abc import Callable
from typing import TYPE_CHECKING, TypeVar

from llmtrain.registry.core import Registry, RegistryError

if TYPE_CHECKING:
    from llmtrain.data.base import DataModule

__all__ = ["RegistryError", "available_data_modules", "get_data_module", "register_data_module"]

D = TypeVar("D")
DATA_MODULES: Registry = Registry("Data module")


def register_data_module(name: str) -> Callable[[type[D]], type[D]]:
    return DATA_MODULES.register(name)


def get_data_module(name: str) -> type[DataModule]:
    return DATA_MODULES.get(name)


def available_data_modules() -> list[str]:
    return DATA_MODULES.names()
