"""Server, backends (native engine / remote vLLM / remote Ollama) and session state."""

from app.core.conversation_manager import ConversationManager
from app.core.ollama_handler import OllamaHandler

__all__ = ["OllamaHandler", "ConversationManager"]
