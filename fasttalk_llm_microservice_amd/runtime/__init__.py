"""Host runtime (C++ `_rt` extension): KV block manager with prefix caching,
incremental UTF-8 detokenizer, JSON-schema token FSM."""
from __future__ import annotations

import os
import threading

_lock = threading.Lock()
_rt = None


def rt():
    global _rt
    if _rt is not None:
        return _rt
    with _lock:
        if _rt is None and os.environ.get("FT_RT_MODULE"):
            # a differently built copy of the same bindings, e.g. the ASan/UBSan
            # executable's embedded module (tests/unit/test_sanitizers.py)
            import importlib

            _rt = importlib.import_module(os.environ["FT_RT_MODULE"])
        if _rt is None:
            try:
                from .. import _rt as mod  # type: ignore
            except ImportError:
                if os.environ.get("FT_AUTOBUILD", "1") == "0":
                    raise
                from ..ops.build import build_runtime

                build_runtime(verbose=True)
                from .. import _rt as mod  # type: ignore
            _rt = mod
    return _rt
