"""Per-session conversation history (API of the reference
``app/core/conversation_manager.py``: ``ConversationState``,
``ConversationManager``; OpenAI-shaped ``{"role", "content"}`` messages, system
prompt kept as message 0 when trimming to ``max_history_length``).

Token-aware truncation (Appendix D Q17) lives in the engine adapter
(:mod:`app.core.native_handler`), which knows the tokenizer and
``max_model_len``; this class keeps the reference's count-based semantics.
"""
from __future__ import annotations

import logging
import time
from dataclasses import dataclass, field
from typing import Any, Dict, List, Optional

from app.core.text_processor import TextContext

logger = logging.getLogger(__name__)


@dataclass
class ConversationState:
    session_id: str
    system_prompt: Optional[str] = None
    messages: List[Dict[str, str]] = field(default_factory=list)
    max_history_length: int = 50
    created_at: float = field(default_factory=time.time)
    last_updated: float = field(default_factory=time.time)
    total_turns: int = 0
    total_tokens_generated: int = 0

    def _has_system(self) -> bool:
        return bool(self.messages) and self.messages[0].get("role") == "system"

    def add_message(self, role: str, content: str):
        self.messages.append({"role": role, "content": content})
        self.total_turns += 1
        self.last_updated = time.time()
        if len(self.messages) > self.max_history_length:
            if self._has_system():
                keep = self.max_history_length - 1
                self.messages = [self.messages[0]] + (self.messages[-keep:] if keep > 0 else [])
            else:
                self.messages = self.messages[-self.max_history_length:]

    def get_messages_for_api(self) -> List[Dict[str, str]]:
        return list(self.messages)

    def clear_history(self, keep_system_prompt: bool = True):
        self.messages = [self.messages[0]] if (keep_system_prompt and self._has_system()) else []

    def get_age(self) -> float:
        return time.time() - self.created_at

    def get_idle_time(self) -> float:
        return time.time() - self.last_updated


class ConversationManager:
    """In-memory session store (single event loop: no locking needed)."""

    def __init__(self, max_history_length: int = 50):
        self.max_history_length = max_history_length
        self.conversations: Dict[str, ConversationState] = {}
        self.text_context_processor = TextContext()

    def create_session(self, session_id: str, system_prompt: Optional[str] = None,
                       max_history_length: Optional[int] = None) -> ConversationState:
        if session_id in self.conversations:
            self.end_session(session_id)
        st = ConversationState(session_id=session_id, system_prompt=system_prompt,
                               max_history_length=max_history_length or self.max_history_length)
        if system_prompt:
            st.add_message("system", system_prompt)
        self.conversations[session_id] = st
        return st

    def get_session(self, session_id: str) -> Optional[ConversationState]:
        return self.conversations.get(session_id)

    def has_session(self, session_id: str) -> bool:
        return session_id in self.conversations

    def add_user_message(self, session_id: str, content: str) -> bool:
        st = self.conversations.get(session_id)
        if st is None:
            logger.error("Cannot add message: session %s not found", session_id)
            return False
        st.add_message("user", content)
        return True

    def add_assistant_message(self, session_id: str, content: str, tokens_generated: int = 0) -> bool:
        st = self.conversations.get(session_id)
        if st is None:
            logger.error("Cannot add message: session %s not found", session_id)
            return False
        st.add_message("assistant", content)
        st.total_tokens_generated += tokens_generated
        return True

    def get_messages_for_generation(self, session_id: str) -> Optional[List[Dict[str, str]]]:
        st = self.conversations.get(session_id)
        return None if st is None else st.get_messages_for_api()

    def clear_history(self, session_id: str, keep_system_prompt: bool = True) -> bool:
        st = self.conversations.get(session_id)
        if st is None:
            return False
        st.clear_history(keep_system_prompt)
        return True

    def end_session(self, session_id: str) -> bool:
        return self.conversations.pop(session_id, None) is not None

    def cleanup_idle_sessions(self, idle_timeout: float = 3600.0) -> int:
        stale = [sid for sid, st in self.conversations.items() if st.get_idle_time() > idle_timeout]
        for sid in stale:
            self.end_session(sid)
        return len(stale)

    def get_session_count(self) -> int:
        return len(self.conversations)

    def get_all_session_ids(self) -> List[str]:
        return list(self.conversations)

    def get_statistics(self) -> Dict[str, Any]:
        return {
            "active_sessions": len(self.conversations),
            "total_turns": sum(s.total_turns for s in self.conversations.values()),
            "total_tokens_generated": sum(s.total_tokens_generated for s in self.conversations.values()),
        }
