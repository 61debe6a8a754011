"""Plugin registries (reference tests/test_registry.py)."""

from __future__ import annotations

import pytest

from llmtrain.data.base import DataModule
from llmtrain.models.base import ModelAdapter
from llmtrain.registry import initialize_registries
from llmtrain.registry.core import Registry, RegistryError
from llmtrain.registry.data import available_data_modules, get_data_module, register_data_module
from llmtrain.registry.models import (
    MODELS,
    available_model_adapters,
    get_model_adapter,
    register_model,
)


def test_builtin_plugins_registered() -> None:
    initialize_registries()
    assert {"gpt", "dummy_gpt"} <= set(available_model_adapters())
    assert {"dummy_text", "hf_text", "synthetic_tokens"} <= set(available_data_modules())
    assert issubclass(get_model_adapter("gpt"), ModelAdapter)
    assert issubclass(get_data_module(" synthetic_tokens "), DataModule)


def test_register_lookup_and_duplicate() -> None:
    @register_model("test_tmp_adapter")
    class _A(ModelAdapter):  # type: ignore[misc]
        def build_model(self, cfg):  # type: ignore[no-untyped-def]
            return None

        def build_tokenizer(self, cfg):  # type: ignore[no-untyped-def]
            return None

        def compute_loss(self, model, batch):  # type: ignore[no-untyped-def]
            return None

    try:
        assert get_model_adapter("test_tmp_adapter") is _A
        with pytest.raises(RegistryError, match="already registered"):
            register_model("test_tmp_adapter")(_A)
    finally:
        MODELS.unregister("test_tmp_adapter")


def test_unknown_names_list_available() -> None:
    initialize_registries()
    with pytest.raises(RegistryError) as info:
        get_model_adapter("nope")
    assert "Available:" in str(info.value) and "gpt" in str(info.value)
    with pytest.raises(RegistryError, match="Unknown data module 'nope'"):
        get_data_module("nope")


def test_empty_names_rejected() -> None:
    with pytest.raises(RegistryError, match="non-empty"):
        register_data_module("   ")
    with pytest.raises(RegistryError):
        get_model_adapter("")


def test_registry_error_is_value_error() -> None:
    assert issubclass(RegistryError, ValueError)
    reg: Registry[int] = Registry("Thing")
    assert reg.names() == [] and "x" not in reg
