"""Tokenizer (E3 in SURVEY.md §2.3).

The reference never tokenizes: vLLM does (``app/core/vllm_handler.py:191-194``
only sees text deltas).  Our engine owns it.  A real checkpoint directory with
``tokenizer.json`` is loaded as is; otherwise (no network, no HF assets in this
environment) we build a deterministic *synthetic Llama-3 tokenizer*:

* 128,000 regular pieces over the byte-level alphabet (every byte is a piece,
  so every string round-trips) + the 256 Llama-3 special tokens at
  128000-128255 (``<|begin_of_text|>`` ... ``<|eot_id|>``, ``<|python_tag|>``)
  -- the exact id layout of Llama-3.1, so the embedding/LM-head shapes and the
  chat template are those of the real model;
* a Unigram model (Viterbi segmentation; all scores equal -> fewest pieces),
  which averages ~3-4 characters per token on English like the real tokenizer.

Detokenization is byte-exact: :meth:`Tokenizer.id_to_bytes` gives the raw bytes
of every id for the incremental UTF-8-safe detokenizer (runtime/detok).
"""
from __future__ import annotations

import functools
import itertools
import os
import random
import string
from typing import Dict, List, Optional, Sequence

LLAMA3_SPECIALS = [
    "<|begin_of_text|>", "<|end_of_text|>", "<|reserved_special_token_0|>",
    "<|reserved_special_token_1|>", "<|finetune_right_pad_id|>", "<|reserved_special_token_2|>",
    "<|start_header_id|>", "<|end_header_id|>", "<|eom_id|>", "<|eot_id|>", "<|python_tag|>",
] + [f"<|reserved_special_token_{i}|>" for i in range(3, 248)]
assert len(LLAMA3_SPECIALS) == 256

NUM_REGULAR = 128000

_COMMON_WORDS = """the of and to in is you that it he was for on are as with his they at be this have
from or one had by word but not what all were we when your can said there use an each which she do how
their if will up other about out many then them these so some her would make like him into time has look
two more write go see number no way could people my than first water been call who oil its now find long
down day did get come made may part hello world assistant user system help question answer please thank
weather today tomorrow time date search web news information tool call function name parameters result
session voice conversation speak talk listen fast model token stream response request message error
good great yes okay sure know think want need tell give take say going right really well just also very
here where why because before after again still never always something anything nothing everything
new old big small high low next last early late open close start end begin finish stop run walk""".split()


@functools.lru_cache(maxsize=1)
def _bytes_to_unicode() -> Dict[int, str]:
    bs = list(range(ord("!"), ord("~") + 1)) + list(range(ord("¡"), ord("¬") + 1)) + \
        list(range(ord("®"), ord("ÿ") + 1))
    cs = bs[:]
    n = 0
    for b in range(256):
        if b not in bs:
            bs.append(b)
            cs.append(256 + n)
            n += 1
    return {b: chr(c) for b, c in zip(bs, cs)}


def _to_bl(s: str) -> str:
    m = _bytes_to_unicode()
    return "".join(m[b] for b in s.encode("utf-8"))


def synthetic_pieces() -> List[str]:
    """Deterministic list of NUM_REGULAR byte-level pieces (ids 0..127999)."""
    b2u = _bytes_to_unicode()
    pieces: List[str] = [b2u[b] for b in range(256)]
    seen = set(pieces)

    def add(s: str):
        p = _to_bl(s)
        if p not in seen and len(pieces) < NUM_REGULAR:
            seen.add(p)
            pieces.append(p)

    lower = string.ascii_lowercase
    upper = string.ascii_uppercase
    for w in _COMMON_WORDS:
        for v in (w, " " + w, w.capitalize(), " " + w.capitalize()):
            add(v)
    for p in ["\n\n", "  ", "    ", "\t", ".\n", ",", ", ", ". ", "!\n", "?\n", ":\n", "...", " -",
              " (", ")", "\")", "\":", "\": ", "{\"", "\"}", "[\"", "\"]", " {", " }", "{}", "[]",
              " \"", "\",", "\", \"", "'s", "'t", "'re", "'ve", "'m", "'ll", "'d", "\n\n\n", " ="]:
        add(p)
    for a in lower + upper:
        add(" " + a)
    for a, b in itertools.product(lower, repeat=2):
        add(a + b)
        add(" " + a + b)
    for a, b in itertools.product(upper, lower):
        add(a + b)
        add(" " + a + b)
    for n in range(1000):
        add(str(n))
        add(f"{n:03d}")
    for a, b, c in itertools.product(lower, repeat=3):
        add(a + b + c)
        add(" " + a + b + c)
    for a, b, c in itertools.product(upper, lower, lower):
        add(" " + a + b + c)
    rng = random.Random(1234)
    quads = ["".join(t) for t in itertools.product(lower, repeat=4)]
    rng.shuffle(quads)
    for q in quads:
        if len(pieces) >= NUM_REGULAR:
            break
        add(" " + q)
        add(q)
    assert len(pieces) == NUM_REGULAR, len(pieces)
    return pieces


def _build_synthetic_hf():
    from tokenizers import AddedToken, Tokenizer, decoders, models, pre_tokenizers

    pieces = synthetic_pieces()
    vocab = [(p, -1.0) for p in pieces]
    tok = Tokenizer(models.Unigram(vocab, unk_id=None, byte_fallback=False))
    tok.pre_tokenizer = pre_tokenizers.ByteLevel(add_prefix_space=False, use_regex=True)
    tok.decoder = decoders.ByteLevel()
    tok.add_special_tokens([AddedToken(s, special=True, normalized=False) for s in LLAMA3_SPECIALS])
    return tok


def _cache_path() -> str:
    base = os.environ.get("FT_CACHE_DIR") or os.path.join(os.path.dirname(os.path.dirname(
        os.path.dirname(os.path.abspath(__file__)))), "build", "cache")
    return os.path.join(base, "synthetic_llama3_tokenizer_v1.json")


@functools.lru_cache(maxsize=4)
def _load_hf(path: Optional[str]):
    from tokenizers import Tokenizer

    if path:
        return Tokenizer.from_file(path)
    cp = _cache_path()
    if os.path.exists(cp):
        try:
            return Tokenizer.from_file(cp)
        except Exception:
            pass
    tok = _build_synthetic_hf()
    try:
        os.makedirs(os.path.dirname(cp), exist_ok=True)
        tmp = cp + f".{os.getpid()}.tmp"
        tok.save(tmp)
        os.replace(tmp, cp)
    except OSError:
        pass
    return tok


class Tokenizer:
    """Thin wrapper exposing what the engine needs (ids, specials, raw bytes)."""

    def __init__(self, path: Optional[str] = None):
        if path and os.path.isdir(path):
            cand = os.path.join(path, "tokenizer.json")
            path = cand if os.path.exists(cand) else None
        self.path = path
        self.hf = _load_hf(path)
        self.vocab_size = self.hf.get_vocab_size(with_added_tokens=True)
        self._special_ids = {}
        for s in LLAMA3_SPECIALS[:11]:
            i = self.hf.token_to_id(s)
            if i is not None:
                self._special_ids[s] = i
        self.bos_id = self._special_ids.get("<|begin_of_text|>", 128000)
        self.eot_id = self._special_ids.get("<|eot_id|>", 128009)
        self.eom_id = self._special_ids.get("<|eom_id|>", 128008)
        self.eos_id = self._special_ids.get("<|end_of_text|>", 128001)
        self.python_tag_id = self._special_ids.get("<|python_tag|>", 128010)
        self.start_header_id = self._special_ids.get("<|start_header_id|>", 128006)
        self.end_header_id = self._special_ids.get("<|end_header_id|>", 128007)
        self.stop_ids = sorted({self.eot_id, self.eom_id, self.eos_id})

    def special(self, name: str) -> int:
        return self._special_ids[name]

    def encode(self, text: str, add_special_tokens: bool = False) -> List[int]:
        return self.hf.encode(text, add_special_tokens=add_special_tokens).ids

    def encode_batch(self, texts: Sequence[str]) -> List[List[int]]:
        return [e.ids for e in self.hf.encode_batch(list(texts), add_special_tokens=False)]

    def decode(self, ids: Sequence[int], skip_special_tokens: bool = True) -> str:
        return self.hf.decode(list(ids), skip_special_tokens=skip_special_tokens)

    @functools.cached_property
    def id_to_bytes(self) -> List[bytes]:
        """Raw bytes of every id (special tokens -> their literal text or b'')."""
        u2b = {c: b for b, c in _bytes_to_unicode().items()}
        out: List[bytes] = [b""] * self.vocab_size
        specials = set(LLAMA3_SPECIALS)
        for piece, i in self.hf.get_vocab(with_added_tokens=True).items():
            if i >= self.vocab_size:
                continue
            if piece in specials:
                out[i] = b""
                continue
            try:
                out[i] = bytes(u2b[c] for c in piece)
            except KeyError:
                out[i] = piece.encode("utf-8")
        return out

    def is_special(self, token_id: int) -> bool:
        return token_id >= NUM_REGULAR if self.path is None else \
            self.hf.id_to_token(token_id) in set(LLAMA3_SPECIALS)


@functools.lru_cache(maxsize=4)
def get_tokenizer(path: Optional[str] = None) -> Tokenizer:
    return Tokenizer(path)
