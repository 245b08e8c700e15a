"""Tracing and fault injection hooks for the engine step loop (SURVEY.md §5:
"optional torch.profiler/rocprof hooks behind FT_PROFILE" and "fault-injection
env hooks (FT_FAULT_*) for tests").

* ``FT_PROFILE=<steps>`` (+ ``FT_PROFILE_SKIP=<steps>``, ``FT_PROFILE_DIR``):
  wraps that many engine steps (after skipping some) in ``torch.profiler`` with
  CPU + GPU activities and writes a Chrome trace (viewable in Perfetto); for
  kernel-level counters use ``rocprofv3 --kernel-trace --stats`` instead.
* ``FT_FAULT_STEP=<n>`` raises inside the n-th engine step (and the
  ``FT_FAULT_REPEAT - 1`` steps after it); ``FT_FAULT_KIND=runtime|oom|device``
  picks a recoverable RuntimeError, a fatal MemoryError, or a RuntimeError with
  the text of a sticky HIP fault (fatal), which exercises the AsyncEngine error
  path and ``/health``.
"""
from __future__ import annotations

import logging
import os
import time
from typing import Optional

log = logging.getLogger("fasttalk.debug")


class StepProfiler:
    def __init__(self):
        self.steps = int(os.environ.get("FT_PROFILE", "0") or 0)
        self.skip = int(os.environ.get("FT_PROFILE_SKIP", "20") or 0)
        self.out_dir = os.environ.get("FT_PROFILE_DIR", "profiles/traces")
        self._n = 0
        self._prof = None

    @property
    def enabled(self) -> bool:
        return self.steps > 0

    def before_step(self):
        if not self.enabled:
            return
        self._n += 1
        if self._n == self.skip + 1 and self._prof is None:
            import torch

            acts = [torch.profiler.ProfilerActivity.CPU]
            if torch.cuda.is_available():
                acts.append(torch.profiler.ProfilerActivity.CUDA)
            self._prof = torch.profiler.profile(activities=acts, record_shapes=False)
            self._prof.__enter__()

    def after_step(self):
        if self._prof is not None and self._n >= self.skip + self.steps:
            self._prof.__exit__(None, None, None)
            os.makedirs(self.out_dir, exist_ok=True)
            path = os.path.join(self.out_dir, f"engine_steps_{int(time.time())}.json")
            self._prof.export_chrome_trace(path)
            log.warning("FT_PROFILE: wrote %d-step trace to %s", self.steps, path)
            self._prof = None
            self.steps = 0


class FaultInjector:
    def __init__(self):
        self.at: Optional[int] = int(os.environ["FT_FAULT_STEP"]) if os.environ.get("FT_FAULT_STEP") else None
        self.kind = os.environ.get("FT_FAULT_KIND", "runtime")
        self.repeat = max(1, int(os.environ.get("FT_FAULT_REPEAT", "1")))
        self._n = 0

    def check(self):
        if self.at is None:
            return
        self._n += 1
        if self.at <= self._n < self.at + self.repeat:
            if self._n == self.at + self.repeat - 1:
                self.at = None
            if self.kind == "oom":
                raise MemoryError("FT_FAULT: injected out-of-memory in engine step")
            if self.kind == "device":
                raise RuntimeError("FT_FAULT: HIP error: an illegal memory access was encountered")
            raise RuntimeError("FT_FAULT: injected failure in engine step")
