"""Configuration, logging, error handling and connection management."""

from app.utils.config import Config
from app.utils.connection_manager import ConnectionInfo, ConnectionManager, ConnectionState
from app.utils.error_handler import (CircuitBreaker, ErrorCategory, ErrorHandler, ErrorSeverity,
                                     LLMServiceError, RetryManager)
from app.utils.logger import StructuredLogger

__all__ = ["Config", "StructuredLogger", "LLMServiceError", "ErrorCategory", "ErrorSeverity",
           "CircuitBreaker", "RetryManager", "ErrorHandler", "ConnectionManager", "ConnectionInfo",
           "ConnectionState"]
