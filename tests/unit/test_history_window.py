"""Engine history window with hysteresis.

``ConversationManager`` trims to ``max_history_length`` messages exactly like the
reference (``/root/reference/app/core/conversation_manager.py:34-53``); past the
cap the API history slides by one message per message, which would change the
token prefix right after the system block every turn.  ``NativeHandler`` keeps
an engine window that is a suffix of the API history and cuts it in chunks, so
the engine's prefix cache keeps matching across turns."""
import random

from app.core.conversation_manager import ConversationManager
from app.core.native_handler import NativeHandler
from fasttalk_llm_microservice_amd.engine.chat_template import ChatTemplate
from fasttalk_llm_microservice_amd.engine.tokenizer import get_tokenizer

BS = 16


class _Cfg:
    max_history_length = 50


class _FakeEngine:
    def __init__(self):
        self.tokenizer = get_tokenizer(None)
        self.template = ChatTemplate(self.tokenizer)
        self.max_model_len = 8192
        self.model_cfg = type("M", (), {"name": "fake"})()


def _lcp(a, b):
    n = 0
    for x, y in zip(a, b):
        if x != y:
            break
        n += 1
    return n


def _simulate(turns, sessions=12, seed=0):
    h = NativeHandler(_Cfg(), engine=_FakeEngine())
    cm = ConversationManager(max_history_length=50)
    rng = random.Random(seed)
    words = "the voice assistant should answer quickly about weather news music travel".split()
    cached = total = 0
    per_turn = []
    prev = {}
    for s in range(sessions):
        cm.create_session(f"s{s}", "You are a helpful voice assistant.")
    for t in range(turns):
        turn_cached = turn_total = 0
        for s in range(sessions):
            sid = f"s{s}"
            cm.add_user_message(sid, " ".join(rng.choice(words) for _ in range(40)) + "?")
            msgs = cm.get_messages_for_generation(sid)
            ids = h.build_prompt(msgs, 128, session_id=sid)
            # the engine's prefix cache holds every earlier prompt + reply in full
            # blocks (the system block is shared by all sessions)
            hit = max([_lcp(ids, p) for p in prev.values()] + [0])
            hit = (hit // BS) * BS
            hit = min(hit, ((len(ids) - 1) // BS) * BS)
            turn_cached += hit
            turn_total += len(ids)
            gen = [rng.randrange(1000, 60000) for _ in range(128)]
            text = " ".join(rng.choice(words) for _ in range(100))
            h._remember_reply(sid, gen, text)
            prev[sid] = ids + gen
            cm.add_assistant_message(sid, text, 128)
            # the window never holds more than the API history (a suffix of it)
            st = h._sessions[sid]
            assert len(st.fps) <= len(cm.get_messages_for_generation(sid))
        per_turn.append(turn_cached / turn_total)
        cached += turn_cached
        total += turn_total
    return cached / total, per_turn


def test_history_window_keeps_prefix_cache_over_40_turns():
    ratio, per_turn = _simulate(40, sessions=50)
    assert ratio >= 0.95, ratio
    # sessions that start together reach their first cut on different turns (the
    # per-session window lead) and cut again on different turns (the jittered keep
    # sizes): no turn re-prefills most of the sessions at once (p99 TTFT)
    low = [t for t, r in enumerate(per_turn) if t > 1 and r < 0.6]
    assert not low, per_turn


def test_window_is_suffix_of_api_history_and_cuts_in_chunks():
    h = NativeHandler(_Cfg(), engine=_FakeEngine())
    cm = ConversationManager(max_history_length=50)
    cm.create_session("a", "sys")
    cuts = 0
    last = None
    for t in range(60):
        cm.add_user_message("a", f"question {t}")
        msgs = cm.get_messages_for_generation("a")
        h.build_prompt(msgs, 64, session_id="a")
        st = h._sessions["a"]
        n = len(st.fps)
        if last is not None and n < last:
            cuts += 1
            assert last - n >= 10  # a chunk, not one message per turn
        last = n
        # the engine window is exactly the tail of what the API would send
        api = msgs
        assert n <= len(api)
        h._remember_reply("a", [5, 6, 7], f"answer {t}")
        cm.add_assistant_message("a", f"answer {t}", 3)
    assert 1 <= cuts <= 4, cuts


class _WarmEngine(_FakeEngine):
    def __init__(self):
        super().__init__()
        self.warm = []

    def prefill_background(self, ids, session_id=None):
        self.warm.append(list(ids))
        self.warm_sessions = getattr(self, "warm_sessions", []) + [session_id]


import pytest


@pytest.mark.parametrize("tools", [None, [{"type": "function", "function": {
    "name": "web_search", "description": "Search the web", "parameters": {"type": "object"}}}]])
def test_cut_window_prefix_is_warmed_one_turn_ahead(tools):
    """The turn before a window cut queues the cut window's known prefix as a
    background prefill; the cut turn's prompt starts with exactly those tokens, so
    it hits the prefix cache instead of re-prefilling the window on its TTFT."""
    eng = _WarmEngine()
    h = NativeHandler(_Cfg(), engine=eng)
    cm = ConversationManager(max_history_length=50)
    rng = random.Random(1)
    words = "the voice assistant should answer quickly about weather news music travel".split()
    cuts = warmed = 0
    for s in range(6):
        sid = f"w{s}"
        cm.create_session(sid, "You are a helpful voice assistant.")
        last_warm = None
        for t in range(60):
            cm.add_user_message(sid, " ".join(rng.choice(words) for _ in range(20)) + "?")
            n_warm = len(eng.warm)
            ids = h.build_prompt(cm.get_messages_for_generation(sid), 128, session_id=sid, tools=tools)
            st = h._sessions[sid]
            if st.reply_fp is None and st.gen_ids == [] and t and len(st.fps) < prev_len:
                cuts += 1
                assert last_warm is not None, f"cut at turn {t} was not warmed"
                assert ids[:len(last_warm)] == last_warm
                assert len(last_warm) > len(ids) // 2
                warmed += 1
            prev_len = len(st.fps) + 2
            last_warm = eng.warm[-1] if len(eng.warm) > n_warm else None
            text = " ".join(rng.choice(words) for _ in range(30))
            h._remember_reply(sid, [rng.randrange(1000, 60000) for _ in range(40)], text)
            cm.add_assistant_message(sid, text, 40)
    assert cuts >= 6 and warmed == cuts, (cuts, warmed)


def test_tool_rounds_continue_the_session_stream_without_becoming_its_state():
    """The agent's guided tool call and its post-tool answer are built on the
    session's token stream (previous prompt + generated ids), so they hit the
    prefix cache, but they do not replace the state the next turn continues."""
    h = NativeHandler(_Cfg(), engine=_FakeEngine())
    cm = ConversationManager(max_history_length=50)
    cm.create_session("t", "sys")
    cm.add_user_message("t", "hello there")
    ids0 = h.build_prompt(cm.get_messages_for_generation("t"), 64, session_id="t")
    gen = [70001, 70002, 70003]                    # generated ids (not a re-tokenization)
    h._remember_reply("t", gen, "hi! how can I help")
    cm.add_assistant_message("t", "hi! how can I help", 3)
    cm.add_user_message("t", "search the news please")
    msgs = cm.get_messages_for_generation("t")
    before = (list(h._sessions["t"].prompt_ids), list(h._sessions["t"].gen_ids))
    stream = ids0 + gen
    g = h.build_prompt(msgs, 64, session_id="t", remember=False)          # guided round
    assert g[:len(stream)] == stream
    call = {"role": "assistant", "content": '{"name": "web_search", "arguments": {"query": "news"}}'}
    tool = {"role": "tool", "content": "stub results"}
    a = h.build_prompt(msgs + [call, tool], 64, session_id="t", remember=False)   # answer round
    assert a[:len(g) - len(h.template.generation_prompt())] == g[:len(g) - len(h.template.generation_prompt())]
    assert (h._sessions["t"].prompt_ids, h._sessions["t"].gen_ids) == before
    # a full re-render (what these rounds used before) diverges at the first reply
    full = h.template.render(msgs)
    assert full[:len(stream)] != stream


def test_chat_template_message_cache_is_transparent():
    """Rendered message ids are cached by (role, text): a re-render gives the same ids,
    callers may mutate what they get back, and the cache stays bounded."""
    from fasttalk_llm_microservice_amd.engine.chat_template import ChatTemplate
    from fasttalk_llm_microservice_amd.engine.tokenizer import get_tokenizer

    t = ChatTemplate(get_tokenizer())
    msgs = [{"role": "system", "content": "be brief"}, {"role": "user", "content": "hello there"},
            {"role": "assistant", "content": "hi"}, {"role": "tool", "content": "result 1"}]
    a = t.render(msgs)
    a2 = t.render(msgs)
    assert a == a2
    ids = t.message_ids(msgs[1])
    ids.append(-1)
    assert t.message_ids(msgs[1])[-1] != -1
    t.MSG_CACHE = 3
    for i in range(10):
        t.message_ids({"role": "user", "content": f"m{i}"})
    assert len(t._msg_cache) <= 3
    assert t.render(msgs) == a
