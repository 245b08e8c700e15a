"""Error taxonomy, classification, circuit breakers and retry (API of the
reference ``app/utils/error_handler.py``).

Changes vs the reference (SURVEY.md §5 failure detection, Appendix D Q11/Q15):
* ``LLMServiceError.to_dict`` additionally carries ``code`` (= category) so
  every WebSocket error frame has a machine-readable code.
* the classifier knows HIP/ROCm failure strings (``hipError*``, ``HIP out of
  memory``, ``rocm``) and maps them to ``ErrorCategory.GPU``.
* the ``generation`` breaker is actually used: the WS server wraps engine
  generation with :meth:`CircuitBreaker.guard` (an async context manager).
"""
from __future__ import annotations

import contextlib
import logging
import time
from collections import deque
from dataclasses import dataclass, field
from enum import Enum
from threading import Lock
from typing import Any, Callable, Dict, Optional, Tuple

logger = logging.getLogger(__name__)


class ErrorCategory(Enum):
    CONNECTION = "connection"
    PROCESSING = "processing"
    RESOURCE = "resource"
    CONFIGURATION = "configuration"
    SYSTEM = "system"
    GPU = "gpu"
    TIMEOUT = "timeout"
    VALIDATION = "validation"


class ErrorSeverity(Enum):
    LOW = "low"
    MEDIUM = "medium"
    HIGH = "high"
    CRITICAL = "critical"


@dataclass
class ErrorInfo:
    category: ErrorCategory
    severity: ErrorSeverity
    message: str
    recoverable: bool
    timestamp: float = field(default_factory=time.time)
    retry_after: Optional[float] = None
    context: Optional[Dict[str, Any]] = None


class LLMServiceError(Exception):
    """Service error with a category, severity and retry hint."""

    def __init__(self, message: str, category: ErrorCategory = ErrorCategory.SYSTEM,
                 severity: ErrorSeverity = ErrorSeverity.MEDIUM, recoverable: bool = True,
                 retry_after: Optional[float] = None):
        super().__init__(message)
        self.message = message
        self.category = category
        self.severity = severity
        self.recoverable = recoverable
        self.retry_after = retry_after

    def to_dict(self) -> Dict[str, Any]:
        return {
            "code": self.category.value,
            "message": self.message,
            "category": self.category.value,
            "severity": self.severity.value,
            "recoverable": self.recoverable,
            "retry_after": self.retry_after,
        }


class CircuitBreakerState(Enum):
    CLOSED = "closed"
    OPEN = "open"
    HALF_OPEN = "half_open"


class CircuitBreaker:
    """Classic three-state breaker: ``failure_threshold`` consecutive failures
    open it for ``timeout`` seconds; then up to ``half_open_max_calls`` trial
    calls decide between closing and re-opening."""

    def __init__(self, name: str, failure_threshold: int = 5, timeout: float = 60.0,
                 half_open_max_calls: int = 1):
        self.name = name
        self.failure_threshold = failure_threshold
        self.timeout = timeout
        self.half_open_max_calls = half_open_max_calls
        self._state = CircuitBreakerState.CLOSED
        self._failures = 0
        self._opened_at: Optional[float] = None
        self._trials = 0
        self._lock = Lock()

    @property
    def state(self) -> CircuitBreakerState:
        with self._lock:
            return self._state

    def _admit(self):
        with self._lock:
            if self._state is CircuitBreakerState.OPEN:
                if self._opened_at is not None and time.time() - self._opened_at >= self.timeout:
                    logger.info("Circuit breaker '%s': OPEN -> HALF_OPEN", self.name)
                    self._state = CircuitBreakerState.HALF_OPEN
                    self._trials = 0
                else:
                    raise LLMServiceError(f"Circuit breaker '{self.name}' is OPEN",
                                          category=ErrorCategory.RESOURCE,
                                          severity=ErrorSeverity.HIGH, recoverable=True,
                                          retry_after=self.timeout)
            if self._state is CircuitBreakerState.HALF_OPEN:
                if self._trials >= self.half_open_max_calls:
                    raise LLMServiceError(f"Circuit breaker '{self.name}' is HALF_OPEN (max calls reached)",
                                          category=ErrorCategory.RESOURCE,
                                          severity=ErrorSeverity.HIGH, recoverable=True,
                                          retry_after=10.0)
                self._trials += 1

    def _on_success(self):
        with self._lock:
            if self._state is CircuitBreakerState.HALF_OPEN:
                logger.info("Circuit breaker '%s': closing (recovered)", self.name)
            self._state = CircuitBreakerState.CLOSED
            self._failures = 0
            self._trials = 0

    def _on_failure(self):
        with self._lock:
            self._failures += 1
            if self._state is CircuitBreakerState.HALF_OPEN or \
                    self._failures >= self.failure_threshold:
                if self._state is not CircuitBreakerState.OPEN:
                    logger.error("Circuit breaker '%s': opening after %d failures", self.name,
                                 self._failures)
                self._state = CircuitBreakerState.OPEN
                self._opened_at = time.time()
                self._trials = 0

    def call(self, func: Callable, *args, **kwargs) -> Any:
        self._admit()
        try:
            result = func(*args, **kwargs)
        except Exception:
            self._on_failure()
            raise
        self._on_success()
        return result

    @contextlib.asynccontextmanager
    async def guard(self):
        """``async with breaker.guard(): ...`` -- the async form of :meth:`call`."""
        self._admit()
        try:
            yield self
        except Exception:
            self._on_failure()
            raise
        self._on_success()

    def reset(self):
        with self._lock:
            self._state = CircuitBreakerState.CLOSED
            self._failures = 0
            self._trials = 0
            self._opened_at = None


class RetryManager:
    @staticmethod
    def retry_with_backoff(func: Callable, max_attempts: int = 3, base_delay: float = 1.0,
                           max_delay: float = 30.0, backoff_factor: float = 2.0,
                           retriable_exceptions: Tuple = (Exception,)) -> Any:
        delay = base_delay
        for attempt in range(1, max_attempts + 1):
            try:
                return func()
            except retriable_exceptions as e:
                if attempt >= max_attempts:
                    logger.error("All %d retry attempts failed", max_attempts)
                    raise
                logger.warning("Attempt %d/%d failed: %s. Retrying in %.1fs", attempt,
                               max_attempts, e, delay)
                time.sleep(delay)
                delay = min(delay * backoff_factor, max_delay)
        raise RuntimeError("unreachable")


_RULES = (
    (("connection", "refused"), ErrorCategory.CONNECTION, ErrorSeverity.HIGH, True),
    (("timeout", "timed out"), ErrorCategory.TIMEOUT, ErrorSeverity.MEDIUM, True),
    (("cuda", "gpu", "out of memory", "hip", "rocm", "hbm"), ErrorCategory.GPU,
     ErrorSeverity.CRITICAL, True),
    (("resource", "capacity"), ErrorCategory.RESOURCE, ErrorSeverity.HIGH, True),
    (("invalid", "validation"), ErrorCategory.VALIDATION, ErrorSeverity.LOW, False),
)


class ErrorHandler:
    """Central error handler: classification, counters, recent history, breakers."""

    def __init__(self, max_error_history: int = 1000):
        self.max_error_history = max_error_history
        self.error_history: deque = deque(maxlen=max_error_history)
        self.error_counts: Dict[ErrorCategory, int] = {c: 0 for c in ErrorCategory}
        self._lock = Lock()
        # names kept from the reference for /stats compatibility
        self.ollama_circuit_breaker = CircuitBreaker("ollama_connection", failure_threshold=3,
                                                     timeout=300.0)
        self.generation_circuit_breaker = CircuitBreaker("generation", failure_threshold=5,
                                                         timeout=120.0)

    def handle_error(self, error: Exception, context: Optional[Dict[str, Any]] = None) -> ErrorInfo:
        if isinstance(error, LLMServiceError):
            cat, sev, rec, msg = error.category, error.severity, error.recoverable, error.message
        else:
            cat, sev, rec = self._categorize_error(error)
            msg = str(error)
        info = ErrorInfo(category=cat, severity=sev, message=msg, recoverable=rec, context=context)
        with self._lock:
            self.error_history.append(info)
            self.error_counts[cat] += 1
        log = logger.error if sev in (ErrorSeverity.HIGH, ErrorSeverity.CRITICAL) else logger.warning
        log("Error handled: [%s] %s", cat.value, msg)
        return info

    def _categorize_error(self, error: Exception) -> Tuple[ErrorCategory, ErrorSeverity, bool]:
        text = str(error).lower()
        for keys, cat, sev, rec in _RULES:
            if any(k in text for k in keys):
                return cat, sev, rec
        return ErrorCategory.PROCESSING, ErrorSeverity.MEDIUM, True

    def get_error_stats(self) -> Dict[str, Any]:
        with self._lock:
            return {
                "total_errors": sum(self.error_counts.values()),
                "by_category": {c.value: n for c, n in self.error_counts.items()},
                "recent_errors": len(self.error_history),
                "circuit_breakers": {
                    "ollama": self.ollama_circuit_breaker.state.value,
                    "generation": self.generation_circuit_breaker.state.value,
                },
            }

    def reset(self):
        with self._lock:
            self.error_history.clear()
            self.error_counts = {c: 0 for c in ErrorCategory}
        self.ollama_circuit_breaker.reset()
        self.generation_circuit_breaker.reset()
