"""A small typed name → class registry shared by the model and data plugin registries.

Semantics (reference ``registry/models.py:13-54``, ``registry/data.py:13-54``): names are
whitespace-stripped and must be non-empty; registering a name twice raises; looking up an
unknown name raises with the sorted list of available names.
"""

from __future__ import annotations

from collections.abc import Callable
from typing import Generic, TypeVar

T = TypeVar("T")


class RegistryError(ValueError):
    """Invalid, duplicate or unknown registry name."""


class Registry(Generic[T]):
    """Maps plugin names to classes; ``kind`` is used in error messages ("Model adapter")."""

    def __init__(self, kind: str) -> None:
        self._kind = kind
        self._entries: dict[str, type[T]] = {}

    @staticmethod
    def normalize(name: str) -> str:
        key = name.strip() if isinstance(name, str) else ""
        if not key:
            raise RegistryError("Registry name must be non-empty.")
        return key

    def _available(self) -> str:
        return ", ".join(sorted(self._entries)) or "none"

    def register(self, name: str) -> Callable[[type[T]], type[T]]:
        key = self.normalize(name)

        def decorator(cls: type[T]) -> type[T]:
            if key in self._entries:
                raise RegistryError(
                    f"{self._kind} '{key}' is already registered. Available: {self._available()}."
                )
            self._entries[key] = cls
            return cls

        return decorator

    def get(self, name: str) -> type[T]:
        key = self.normalize(name)
        try:
            return self._entries[key]
        except KeyError:
            raise RegistryError(
                f"Unknown {self._kind.lower()} '{key}'. Available: {self._available()}."
            ) from None

    def names(self) -> list[str]:
        return sorted(self._entries)

    def unregister(self, name: str) -> None:
        """Remove an entry (test helper for ad-hoc plugins)."""
        self._entries.pop(self.normalize(name), None)

    def __contains__(self, name: object) -> bool:
        return isinstance(name, str) and name.strip() in self._entries
