"""llmtrain — MI355X-native GPT training framework.

Same user-facing contracts as the reference ``llmtrain`` package (CLI, config schema, plugin
registries, run-directory and checkpoint layout); the compute path is PyTorch-ROCm with
hand-written CDNA4 (gfx950) HIP kernels (``llmtrain.ops``) and RCCL-over-xGMI data parallelism
(``llmtrain.parallel``).
"""

from importlib import metadata

__all__ = ["__version__"]

try:
    __version__ = metadata.version("llmtrain-mi355x")
except metadata.PackageNotFoundError:
    __version__ = "1.2.0+mi355x"
