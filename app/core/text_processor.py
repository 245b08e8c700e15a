"""TTS-friendly text segmentation helpers (API of the reference
``app/core/text_processor.py``: ``TextContext.get_context`` and
``calculate_text_similarity``).  The WS server can use ``TextContext`` to
coalesce token deltas into speakable phrases (``sentence`` streaming mode)."""
from __future__ import annotations

from typing import Iterable, Optional, Set, Tuple

DEFAULT_SPLIT_TOKENS = frozenset({".", "!", "?", ",", ";", ":", "\n", "-", "。", "、"})


class TextContext:
    """Finds the shortest speakable prefix: it must end on a split token, be at
    least ``min_len`` characters and contain ``min_alnum_count`` alphanumerics,
    and is searched within the first ``max_len`` characters."""

    def __init__(self, split_tokens: Optional[Iterable[str]] = None):
        self.split_tokens: Set[str] = set(DEFAULT_SPLIT_TOKENS if split_tokens is None else split_tokens)

    def get_context(self, txt: str, min_len: int = 6, max_len: int = 120,
                    min_alnum_count: int = 10) -> Tuple[Optional[str], Optional[str]]:
        alnum = 0
        limit = min(len(txt), max_len)
        for end in range(1, limit + 1):
            ch = txt[end - 1]
            alnum += ch.isalnum()
            if ch in self.split_tokens and end >= min_len and alnum >= min_alnum_count:
                return txt[:end], txt[end:]
        return None, None


def calculate_text_similarity(text1: str, text2: str) -> float:
    """Jaccard similarity of the lower-cased word sets (0.0 when either is empty)."""
    a = set(text1.lower().split())
    b = set(text2.lower().split())
    if not a or not b:
        return 0.0
    return len(a & b) / len(a | b)
