"""Grammar-constrained decoding (logits processors).

* :class:`JsonGrammar` — any syntactically valid JSON value (Ollama ``format:"json"``
  and JSON-schema ``format`` requests).  A character-level pushdown automaton is
  run over candidate token texts; per-automaton-state results are memoised.
* :class:`ToolCallGrammar` — the agents' tool-call language (one JSON object with an
  ``action`` from the tool list and the fields that tool takes, k8s-name-shaped
  strings, integer replicas; ``Minimal_RAG/Program.cs:137-148``).  Random-init
  weights never produce a valid tool call on their own; with this processor every
  request exercises the real dispatch / gating path end-to-end.

A processor is ``callable(generated_ids) -> list[int] | None`` (allowed next ids).
"""
from __future__ import annotations

import re
from typing import Optional

WS = " \t\n\r"


# ----------------------------------------------------------------------------- JSON PDA
class _J:
    """Immutable JSON prefix-automaton state: (mode, stack, aux)."""

    __slots__ = ()

    # modes
    VALUE, OBJ_FIRST, OBJ_KEY, COLON, OBJ_NEXT, ARR_FIRST, ARR_NEXT, STR, ESC, UHEX, NUM, LIT, DONE = range(13)


def _after_value(stack):
    if not stack:
        return (_J.DONE, stack, None)
    return (_J.OBJ_NEXT if stack[-1] == "{" else _J.ARR_NEXT, stack, None)


def _num_ok(s: str, final: bool) -> bool:
    full = re.fullmatch(r"-?(0|[1-9]\d*)(\.\d+)?([eE][+-]?\d+)?", s)
    if final:
        return full is not None
    return full is not None or re.fullmatch(r"-?((0|[1-9]\d*)(\.(\d+([eE][+-]?\d*)?)?|[eE][+-]?\d*)?)?", s) is not None


def json_feed(st, ch):
    mode, stack, aux = st
    if mode == _J.DONE:
        return st if ch in WS else None
    if mode == _J.STR:
        key = aux
        if ch == '"':
            if key:
                return (_J.COLON, stack, None)
            return _after_value(stack)
        if ch == "\\":
            return (_J.ESC, stack, key)
        if ord(ch) < 0x20:
            return None
        return st
    if mode == _J.ESC:
        if ch in '"\\/bfnrt':
            return (_J.STR, stack, aux)
        if ch == "u":
            return (_J.UHEX, stack, (aux, 0))
        return None
    if mode == _J.UHEX:
        key, n = aux
        if ch not in "0123456789abcdefABCDEF":
            return None
        return (_J.STR, stack, key) if n == 3 else (_J.UHEX, stack, (key, n + 1))
    if mode == _J.NUM:
        if ch in "0123456789+-.eE":
            s = aux + ch
            return (_J.NUM, stack, s) if _num_ok(s, False) else None
        if not _num_ok(aux, True):
            return None
        return json_feed(_after_value(stack), ch)
    if mode == _J.LIT:
        rest = aux
        if ch != rest[0]:
            return None
        return (_J.LIT, stack, rest[1:]) if len(rest) > 1 else _after_value(stack)
    if ch in WS:
        return st
    if mode in (_J.VALUE, _J.ARR_FIRST):
        if mode == _J.ARR_FIRST and ch == "]":
            return _after_value(stack[:-1])
        if ch == "{":
            return (_J.OBJ_FIRST, stack + ("{",), None)
        if ch == "[":
            return (_J.ARR_FIRST, stack + ("[",), None)
        if ch == '"':
            return (_J.STR, stack, False)
        if ch in "-0123456789":
            return (_J.NUM, stack, ch)
        for lit in ("true", "false", "null"):
            if ch == lit[0]:
                return (_J.LIT, stack, lit[1:])
        return None
    if mode in (_J.OBJ_FIRST, _J.OBJ_KEY):
        if ch == '"':
            return (_J.STR, stack, True)
        if mode == _J.OBJ_FIRST and ch == "}":
            return _after_value(stack[:-1])
        return None
    if mode == _J.COLON:
        return (_J.VALUE, stack, None) if ch == ":" else None
    if mode == _J.OBJ_NEXT:
        if ch == ",":
            return (_J.OBJ_KEY, stack, None)
        if ch == "}":
            return _after_value(stack[:-1])
        return None
    if mode == _J.ARR_NEXT:
        if ch == ",":
            return (_J.VALUE, stack, None)
        if ch == "]":
            return _after_value(stack[:-1])
        return None
    return None


def json_feed_text(st, text):
    for ch in text:
        st = json_feed(st, ch)
        if st is None:
            return None
    return st


JSON_START = (_J.VALUE, (), None)


class _TokenTable:
    """Decoded text of every token + cheap classes (cached per tokenizer)."""

    _cache: dict = {}

    def __init__(self, tok):
        self.texts = [tok.piece(i) for i in range(tok.vocab_size)]
        self.eos = sorted(tok.eos_ids)
        # tokens usable inside a JSON string without escapes
        self.plain_str = [i for i, t in enumerate(self.texts)
                          if t and '"' not in t and "\\" not in t and all(ord(c) >= 0x20 for c in t)
                          and "�" not in t and i not in tok.eos_ids]
        plain = set(self.plain_str)
        self.special = [i for i, t in enumerate(self.texts) if t and i not in plain
                        and i not in tok.eos_ids and "�" not in t]

    @classmethod
    def get(cls, tok):
        k = id(tok)
        if k not in cls._cache:
            cls._cache[k] = cls(tok)
        return cls._cache[k]


class JsonGrammar:
    def __init__(self, tok, max_cache: int = 4096):
        self.tok = tok
        self.tt = _TokenTable.get(tok)
        self.cache: dict = {}
        self.max_cache = max_cache

    def state_after(self, ids: list):
        st = JSON_START
        text = self.tok.decode(ids) if ids else ""
        return json_feed_text(st, text)

    def allowed(self, st) -> list:
        if st is None:
            return self.tt.eos or [0]
        hit = self.cache.get(st)
        if hit is not None:
            return hit
        mode = st[0]
        texts = self.tt.texts
        if mode == _J.DONE:
            out = list(self.tt.eos) or [0]
        elif mode == _J.STR:
            out = list(self.tt.plain_str) + [i for i in self.tt.special if json_feed_text(st, texts[i]) is not None]
        else:
            cand = range(len(texts))
            out = [i for i in cand if texts[i] and i not in self.tt.eos and "�" not in texts[i]
                   and json_feed_text(st, texts[i]) is not None]
        if len(self.cache) < self.max_cache:
            self.cache[st] = out
        return out

    def __call__(self, ids: list):
        return self.allowed(self.state_after(ids))


def json_logits_processor(tok, schema: Optional[dict] = None):
    """``format: "json"`` / schema -> a JSON constraint (schema keys are not enforced
    beyond syntactic validity)."""
    return JsonGrammar(tok)


# ----------------------------------------------------------------------------- tool calls
K8S_CHARS = set("abcdefghijklmnopqrstuvwxyz0123456789-.")

TOOL_FIELDS = {
    "list_pods": [("namespace", "str")],
    "get_logs": [("namespace", "str"), ("pod", "str")],
    "scale_deployment": [("namespace", "str"), ("name", "str"), ("replicas", "int")],
    "cluster_context": [],
    "final_answer": [],
}


class ToolCallGrammar:
    """Constrains output to ``{"action":"<tool>"[,"field":...]}``.  Fields per tool from
    TOOL_FIELDS; strings are k8s names (``[a-z0-9-.]{1,max_str}``), ints 1-2 digits."""

    def __init__(self, tok, tools: Optional[dict] = None, max_str: int = 24, enums: Optional[dict] = None):
        self.tok = tok
        self.tools = tools or TOOL_FIELDS
        self.max_str = max_str
        # field name -> allowed string values (e.g. namespace -> the RAG allowlist), or a dict
        # {"__by__": earlier field, value of that field: [values]} (e.g. pod names per namespace)
        self.enums = {k: (dict(v) if isinstance(v, dict) else list(v)) for k, v in (enums or {}).items()}
        self.tt = _TokenTable.get(tok)
        texts = self.tt.texts
        self.name_tokens = [i for i, t in enumerate(texts) if t and set(t) <= K8S_CHARS]
        self.digit_tokens = [i for i, t in enumerate(texts) if t and t.isdigit() and len(t) <= 2]
        self.by_text: dict[str, list] = {}
        for i, t in enumerate(texts):
            if t and i not in self.tt.eos:
                self.by_text.setdefault(t, []).append(i)
        self._prefix_cache: dict[str, list] = {}
        # id(history list) -> (list, length, last id, decoded text): a running request's text is
        # extended by its new tokens' texts instead of re-decoding the whole history every step
        # (~17 us per row per step at 128 rows; the host builds the masks while the device waits)
        self._texts: dict = {}
        self._eos = set(self.tt.eos)
        # (kind, room, value state, closing literal) -> allowed ids of a free string / int
        # field (a few dozen keys; building one scans the vocabulary subset, ~1 ms)
        self._free_cache: dict = {}

    def _free_tokens(self, kind: str, room: int, val: str, close: Optional[str]):
        toks = self.name_tokens if kind == "str" else self.digit_tokens
        allowed = [i for i in toks if len(self.tt.texts[i]) <= room] if room > 0 else []
        if kind == "int":  # JSON integers: no leading zero ("0" alone is fine)
            if val == "0":
                allowed = []
            elif not val:
                allowed = [i for i in allowed if self.tt.texts[i] == "0" or self.tt.texts[i][0] != "0"]
        if close is not None:
            allowed = allowed + self._literal_tokens(close)
        return allowed or list(self.tt.eos or [0])

    def _choice(self, options: tuple, typed: str) -> list:
        """Tokens continuing ``typed`` towards any of ``options`` + closing quote (cached)."""
        key = (options, typed)
        c = self._free_cache.get(key)
        if c is None:
            out = set()
            for a in options:
                if a.startswith(typed):
                    out.update(self._literal_tokens((a + '"')[len(typed):]))
            c = sorted(out) or list(self.tt.eos or [0])
            if len(self._free_cache) < 8192:
                self._free_cache[key] = c
        return c

    def _enum_values(self, name: str, before: str) -> list:
        """Allowed values of enum field ``name``; a per-key dict picks the list of the value
        the object already gave its ``__by__`` field (no list for it: no valid value)."""
        vals = self.enums[name]
        if not isinstance(vals, dict):
            return vals
        m = re.search(r'"%s":"([^"]*)"' % re.escape(vals.get("__by__", "")), before)
        return list(vals.get(m.group(1), ())) if m else []

    def _literal_tokens(self, rest: str) -> list:
        """Tokens for a forced literal: those spelling the LONGEST prefix of ``rest`` the
        vocabulary has (the canonical tokenisation a tokenizer would produce; a forced
        literal is not a choice, so fast-forwarding it keeps calls short)."""
        c = self._prefix_cache.get(rest)
        if c is None:
            c = []
            for k in range(len(rest), 0, -1):
                c = list(self.by_text.get(rest[:k], ()))
                if c:
                    break
            if len(self._prefix_cache) < 8192:
                self._prefix_cache[rest] = c
        return c

    def _expand(self, action: Optional[str]):
        """Program for the given action: list of ('lit', s) / ('str',) / ('int',)."""
        prog = [("lit", '{"action":"')]
        if action is None:
            return prog
        prog.append(("lit", action + '"'))
        for name, kind in self.tools[action]:
            prog.append(("lit", f',"{name}":' + ('"' if kind == "str" else "")))
            if kind == "str" and name in self.enums:
                prog.append(("enum", name))
                continue  # the enum step consumes its closing quote
            prog.append((kind,))
            if kind == "str":
                prog.append(("lit", '"'))
        prog.append(("lit", "}"))
        return prog

    def _text(self, ids: list) -> str:
        """decode(ids), incrementally for an append-only history: printable-ASCII token texts
        concatenate exactly (byte-level BPE), end-of-sequence ids decode to nothing; anything
        else (or a history that changed other than by appending) re-decodes in full."""
        n = len(ids)
        if n == 0:
            return ""
        hit = self._texts.get(id(ids))
        if hit is not None and hit[0] is ids and 0 < hit[1] <= n and ids[hit[1] - 1] == hit[2]:
            texts, add = self.tt.texts, []
            for t in ids[hit[1]:]:
                if t in self._eos:
                    continue
                piece = texts[t] if 0 <= t < len(texts) else None
                if not piece or not piece.isascii() or not piece.isprintable():
                    add = None
                    break
                add.append(piece)
            if add is not None:
                text = hit[3] + "".join(add)
                self._texts[id(ids)] = (ids, n, ids[-1], text)
                return text
        text = self.tok.decode(ids)
        if len(self._texts) > 8192:
            self._texts.clear()
        self._texts[id(ids)] = (ids, n, ids[-1], text)
        return text

    def __call__(self, ids: list):
        text = self._text(ids) if ids else ""
        head = '{"action":"'
        if not head.startswith(text[: len(head)]) and not text.startswith(head):
            return self.tt.eos or [0]
        if len(text) < len(head):
            return self._literal_tokens(head[len(text):])
        rest = text[len(head):]
        q = rest.find('"')
        if q < 0:  # choosing the tool name
            return self._choice(tuple(self.tools), rest)
        action = rest[:q]
        if action not in self.tools:
            return self.tt.eos or [0]
        prog = self._expand(action)[1:]
        pos = len(head)
        s = text
        for si, step in enumerate(prog):
            if step[0] == "lit":
                lit = step[1] if step[1] != action + '"' else action + '"'
                seg = s[pos:pos + len(lit)]
                if len(seg) < len(lit):
                    if not lit.startswith(seg):
                        return self.tt.eos or [0]
                    return self._literal_tokens(lit[len(seg):])
                if seg != lit:
                    return self.tt.eos or [0]
                pos += len(lit)
            elif step[0] == "enum":
                vals = self._enum_values(step[1], s[:pos])
                seg = s[pos:]
                q2 = seg.find('"')
                if q2 < 0:  # still choosing the value
                    return self._choice(tuple(vals), seg)
                if seg[:q2] not in vals:
                    return self.tt.eos or [0]
                pos += q2 + 1
            else:
                kind = step[0]
                m = re.match(r"[a-z0-9\-.]*" if kind == "str" else r"\d*", s[pos:])
                val = m.group(0)
                after = s[pos + len(val):]
                limit = self.max_str if kind == "str" else 2
                if after == "":
                    close = prog[si + 1][1] if val else None  # may close the field
                    key = (kind, limit - len(val), "0" if val == "0" else bool(val), close)
                    allowed = self._free_cache.get(key)
                    if allowed is None:
                        allowed = self._free_tokens(kind, limit - len(val), val, close)
                        self._free_cache[key] = allowed
                    return allowed
                if not val:
                    return self.tt.eos or [0]
                pos += len(val)
        return self.tt.eos or [0]  # complete object -> only EOS


def tool_call_processor(tok, tools: Optional[dict] = None, max_str: int = 24, enums: Optional[dict] = None):
    return ToolCallGrammar(tok, tools, max_str, enums)
