"""Voice agent with tool calling."""

from app.agents.voice_agent import ConversationContext, VoiceAgent

__all__ = ["VoiceAgent", "ConversationContext"]
