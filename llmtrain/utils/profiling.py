"""Step-window profiling (the reference has no tracing at all).

``trainer.extra.profile = {"start_step": 5, "steps": 3}`` wraps those optimizer steps in
``torch.profiler`` (ROCm: roctracer/rocprofiler activity for every HIP kernel, including the
``llmtrain_hip`` custom kernels under their own names) and writes a Chrome trace plus a
kernel-time table to ``<run_dir>/profile/``.  For hardware counters use ``rocprofv3`` on the
command line (``scripts/profile.sh``).
"""

from __future__ import annotations

import logging
from pathlib import Path
from typing import Any

import torch

__all__ = ["StepProfiler"]

logger = logging.getLogger(__name__)


class StepProfiler:
    def __init__(self, spec: dict[str, Any] | bool, out_dir: Path) -> None:
        spec = spec if isinstance(spec, dict) else {}
        self.start = int(spec.get("start_step", 3))
        self.stop = self.start + int(spec.get("steps", 2))
        self.out_dir = out_dir
        self._prof: Any = None

    def before_step(self, step: int) -> None:
        if step == self.start and self._prof is None:
            activities = [torch.profiler.ProfilerActivity.CPU]
            if torch.cuda.is_available():
                activities.append(torch.profiler.ProfilerActivity.CUDA)
            self._prof = torch.profiler.profile(activities=activities, record_shapes=False)
            self._prof.__enter__()

    def after_step(self, step: int) -> None:
        if self._prof is not None and step + 1 >= self.stop:
            self.close()

    def close(self) -> None:
        if self._prof is None:
            return
        if torch.cuda.is_available():
            torch.cuda.synchronize()
        self._prof.__exit__(None, None, None)
        self.out_dir.mkdir(parents=True, exist_ok=True)
        trace = self.out_dir / "trace.json"
        self._prof.export_chrome_trace(str(trace))
        sort_key = "self_cuda_time_total" if torch.cuda.is_available() else "self_cpu_time_total"
        table = self._prof.key_averages().table(sort_by=sort_key, row_limit=40)
        (self.out_dir / "kernels.txt").write_text(table, encoding="utf-8")
        logger.info("profiler: wrote %s", trace)
        self._prof = None
