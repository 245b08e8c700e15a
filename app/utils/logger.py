"""Structured logging (API of the reference ``app/utils/logger.py``:
``StructuredLogger``, ``JsonFormatter``, ``ConsoleFormatter``, ``get_logger``,
``request_context``).

Fixes Appendix D Q10: records go through ``Logger.log`` so ``LOG_LEVEL`` is
honoured, and the named loggers do not propagate to the root handler
(``main.py``'s ``basicConfig``), so lines are not printed twice.
"""
from __future__ import annotations

import json
import logging
import os
import sys
from contextvars import ContextVar
from datetime import datetime, timezone
from typing import Any, Dict, Optional

request_context: ContextVar[Optional[str]] = ContextVar("request_context", default=None)

_LEVELS = {"DEBUG": logging.DEBUG, "INFO": logging.INFO, "WARNING": logging.WARNING,
           "WARN": logging.WARNING, "ERROR": logging.ERROR, "CRITICAL": logging.CRITICAL}


def _level(name: Optional[str]) -> int:
    return _LEVELS.get(str(name or "INFO").upper(), logging.INFO)


class JsonFormatter(logging.Formatter):
    """One JSON object per record (log aggregation friendly)."""

    def format(self, record: logging.LogRecord) -> str:
        doc: Dict[str, Any] = {
            "timestamp": datetime.now(timezone.utc).isoformat(),
            "level": record.levelname,
            "service": "llm-service",
            "component": record.name,
            "message": record.getMessage(),
        }
        rid = request_context.get()
        if rid:
            doc["request_id"] = rid
        if record.exc_info:
            doc["exception"] = self.formatException(record.exc_info)
        extra = getattr(record, "extra_fields", None)
        if extra:
            doc.update(extra)
        return json.dumps(doc, default=str)


class ConsoleFormatter(logging.Formatter):
    """``time | LEVEL | component | message`` with ANSI colour per level."""

    COLORS = {"DEBUG": "\033[36m", "INFO": "\033[32m", "WARNING": "\033[33m",
              "ERROR": "\033[31m", "CRITICAL": "\033[35m", "RESET": "\033[0m"}

    def format(self, record: logging.LogRecord) -> str:
        c = self.COLORS.get(record.levelname, self.COLORS["RESET"])
        ts = datetime.now(timezone.utc).strftime("%Y-%m-%d %H:%M:%S")
        msg = record.getMessage()
        rid = request_context.get()
        if rid:
            msg = f"[{rid[:8]}] {msg}"
        line = f"{ts} | {c}{record.levelname:8s}{self.COLORS['RESET']} | {record.name:30s} | {msg}"
        if record.exc_info:
            line += "\n" + self.formatException(record.exc_info)
        return line


class StructuredLogger:
    """Logger wrapper: kwargs become structured ``extra_fields``."""

    def __init__(self, name: str, log_level: str = "INFO", log_file: Optional[str] = None,
                 enable_console: bool = True, enable_file: bool = True):
        self.logger = logging.getLogger(name)
        self.logger.setLevel(_level(log_level))
        self.logger.propagate = False
        for h in list(self.logger.handlers):
            self.logger.removeHandler(h)
        if enable_console:
            h = logging.StreamHandler(sys.stdout)
            h.setFormatter(ConsoleFormatter())
            self.logger.addHandler(h)
        if enable_file and log_file:
            os.makedirs(os.path.dirname(os.path.abspath(log_file)), exist_ok=True)
            fh = logging.FileHandler(log_file)
            fh.setFormatter(JsonFormatter())
            self.logger.addHandler(fh)

    # context -----------------------------------------------------------------
    def set_request_context(self, request_id: str):
        request_context.set(request_id)

    def clear_request_context(self):
        request_context.set(None)

    # levels -------------------------------------------------------------------
    def _emit(self, level: int, message: str, kwargs: Dict[str, Any]):
        if not self.logger.isEnabledFor(level):
            return
        exc_info = kwargs.pop("exc_info", None)
        extra = {"extra_fields": kwargs} if kwargs else None
        self.logger.log(level, message, exc_info=exc_info, extra=extra)

    def debug(self, message: str, **kwargs):
        self._emit(logging.DEBUG, message, kwargs)

    def info(self, message: str, **kwargs):
        self._emit(logging.INFO, message, kwargs)

    def warning(self, message: str, **kwargs):
        self._emit(logging.WARNING, message, kwargs)

    def error(self, message: str, **kwargs):
        self._emit(logging.ERROR, message, kwargs)

    def critical(self, message: str, **kwargs):
        self._emit(logging.CRITICAL, message, kwargs)

    def exception(self, message: str, **kwargs):
        kwargs.setdefault("exc_info", True)
        self._emit(logging.ERROR, message, kwargs)

    # domain helpers -------------------------------------------------------------
    def log_generation(self, prompt: str, tokens_generated: int, processing_time: float,
                       tokens_per_second: float, model: str):
        preview = prompt if len(prompt) <= 100 else prompt[:100] + "..."
        self.info(f"Generation complete: {tokens_generated} tokens in {processing_time:.2f}s "
                  f"({tokens_per_second:.1f} tok/s)", prompt_preview=preview,
                  tokens_generated=tokens_generated, processing_time_seconds=processing_time,
                  tokens_per_second=tokens_per_second, model=model)

    def log_performance(self, component: str, operation: str, duration: float, **kwargs):
        self.info(f"Performance: {component}.{operation} took {duration:.4f}s", component=component,
                  operation=operation, duration_seconds=duration, **kwargs)

    def log_connection(self, session_id: str, action: str, **kwargs):
        self.info(f"Connection {action}: {session_id}", session_id=session_id, action=action,
                  **kwargs)


def get_logger(name: str, log_level: Optional[str] = None,
               log_file: Optional[str] = None) -> StructuredLogger:
    level = log_level or os.getenv("LOG_LEVEL", "INFO")
    log_file = log_file or os.getenv("LOG_FILE") or None
    return StructuredLogger(name, level, log_file, enable_console=True,
                            enable_file=log_file is not None)
