"""System.Text.Json compatibility (.NET 9 defaults), SURVEY §A.2.

Serializer (``JsonSerializer.Serialize`` with default options): compact, member
names as given, ``JavaScriptEncoder.Default`` escaping — everything outside Basic
Latin plus ``" & ' + < > \\` `` and control characters as upper-case ``\\uXXXX``
(``\\b \\t \\n \\f \\r \\\\`` keep their short forms), doubles in shortest round-trip
form with .NET exponent style (``1E-05``).

Deserializer (``JsonSerializer.Deserialize<T>`` with ``PropertyNameCaseInsensitive``):
strict RFC 8259 (no NaN / comments / trailing commas / trailing content), root must
be an object (or ``null``), typed fields: strings must be JSON strings, ``int?`` must
be an integer literal in Int32 range — a quoted number raises (the reason the
``"replicas":"NUM"`` exemplar of ``Minimal_Agent_RAG/Program.cs:44`` breaks, quirk A.7.2).
"""
from __future__ import annotations

import json
import math
import re
from typing import Any, Optional

_SHORT = {"\b": "\\b", "\t": "\\t", "\n": "\\n", "\f": "\\f", "\r": "\\r", "\\": "\\\\"}
_ESC_ASCII = set('"&\'+<>`') | {chr(0x7F)}


def _esc_char(ch: str) -> str:
    if ch in _SHORT:
        return _SHORT[ch]
    o = ord(ch)
    if o > 0xFFFF:
        o -= 0x10000
        return "\\u%04X\\u%04X" % (0xD800 + (o >> 10), 0xDC00 + (o & 0x3FF))
    return "\\u%04X" % o


# everything JavaScriptEncoder.Default escapes: controls, the HTML-sensitive ASCII set,
# DEL and all non-ASCII; runs of safe characters pass through re.sub untouched (C speed)
_NEEDS_ESC = re.compile("[\x00-\x1f\\\\\"&'+<>`\x7f-\U0010ffff]")
_ESC_CACHE: dict = {}


def _esc_sub(m) -> str:
    ch = m.group(0)
    r = _ESC_CACHE.get(ch)
    if r is None:
        r = _ESC_CACHE[ch] = _esc_char(ch)
    return r


def _esc_str(s: str) -> str:
    return '"' + _NEEDS_ESC.sub(_esc_sub, s) + '"'


def _esc_str_slow(s: str) -> str:
    """Character-by-character reference form of :func:`_esc_str` (tests)."""
    out = ['"']
    for ch in s:
        o = ord(ch)
        if ch in _SHORT or o < 0x20 or ch in _ESC_ASCII or o > 0x7E:
            out.append(_esc_char(ch))
        else:
            out.append(ch)
    out.append('"')
    return "".join(out)


def _num(x) -> str:
    if isinstance(x, bool):
        return "true" if x else "false"
    if isinstance(x, int):
        return str(x)
    if math.isnan(x) or math.isinf(x):
        raise ValueError(".NET cannot serialize NaN/Infinity by default")
    r = repr(float(x))
    if r.endswith(".0") and "e" not in r:
        r = r[:-2]
    if "e" in r:
        m, e = r.split("e")
        if m.endswith(".0"):
            m = m[:-2]
        sign = "-" if e.startswith("-") else "+"
        e = e.lstrip("+-").lstrip("0")
        r = f"{m}E{sign}{e.zfill(2)}"
    return r


def dumps(obj: Any) -> str:
    if obj is None:
        return "null"
    if isinstance(obj, bool):
        return "true" if obj else "false"
    if isinstance(obj, (int, float)):
        return _num(obj)
    if isinstance(obj, str):
        return _esc_str(obj)
    if isinstance(obj, dict):
        return "{" + ",".join(_esc_str(str(k)) + ":" + dumps(v) for k, v in obj.items()) + "}"
    if isinstance(obj, (list, tuple)):
        return "[" + ",".join(dumps(v) for v in obj) + "]"
    if hasattr(obj, "__dict__"):
        return dumps(vars(obj))
    raise TypeError(f"cannot serialize {type(obj)}")


class NetJsonError(ValueError):
    """Mirrors System.Text.Json.JsonException (message shaped like .NET's)."""


def _pos(text: str, idx: int) -> tuple[int, int]:
    line = text.count("\n", 0, idx)
    col = idx - (text.rfind("\n", 0, idx) + 1)
    return line, col


def _reject_constant(name):
    raise NetJsonError(f"'{name[0]}' is an invalid start of a value.")


def loads_strict(text: str) -> Any:
    if text is None:
        raise NetJsonError("The input does not contain any JSON tokens.")
    s = text
    stripped = s.strip(" \t\r\n")
    if not stripped:
        raise NetJsonError("The input does not contain any JSON tokens. Expected the input to start with a "
                           "valid JSON token, while the final block is 'true'. Path: $ | LineNumber: 0 | "
                           "BytePositionInLine: 0.")
    try:
        dec = json.JSONDecoder(parse_constant=_reject_constant, strict=True)
        start = len(s) - len(s.lstrip(" \t\r\n"))
        val, end = dec.raw_decode(s, start)
    except NetJsonError as e:
        raise NetJsonError(f"{e} Path: $ | LineNumber: 0 | BytePositionInLine: 0.")
    except json.JSONDecodeError as e:
        ch = s[e.pos] if e.pos < len(s) else ""
        line, col = _pos(s, e.pos)
        if e.pos == len(s) - len(s.lstrip(" \t\r\n")):
            raise NetJsonError(f"'{ch}' is an invalid start of a value. Path: $ | LineNumber: {line} | "
                               f"BytePositionInLine: {col}.")
        raise NetJsonError(f"'{ch}' is invalid after a value. Expected either ',', '}}', or ']'. Path: $ | "
                           f"LineNumber: {line} | BytePositionInLine: {col}.")
    rest = s[end:]
    if rest.strip(" \t\r\n"):
        i = end + (len(rest) - len(rest.lstrip(" \t\r\n")))
        line, col = _pos(s, i)
        raise NetJsonError(f"'{s[i]}' is invalid after a single JSON value. Expected end of data. Path: $ | "
                           f"LineNumber: {line} | BytePositionInLine: {col}.")
    return val


_INT_RE = re.compile(r"-?(0|[1-9]\d*)$")


def _typed(obj: dict, name: str, kind: str):
    """Case-insensitive member lookup (last duplicate wins) with .NET type rules."""
    val, found = None, False
    for k, v in obj.items():
        if k.lower() == name.lower():
            val, found = v, True
    if not found or val is None:
        return None
    if kind == "string":
        if not isinstance(val, str):
            raise NetJsonError(f"The JSON value could not be converted to System.String. Path: $.{name} | "
                               "LineNumber: 0 | BytePositionInLine: 0.")
        return val
    if kind == "int":
        if isinstance(val, bool) or not isinstance(val, int) or not (-2**31 <= val < 2**31):
            raise NetJsonError("The JSON value could not be converted to System.Nullable`1[System.Int32]. "
                               f"Path: $.{name} | LineNumber: 0 | BytePositionInLine: 0.")
        return val
    raise ValueError(kind)


def _int_literals_ok(text: str, obj) -> None:
    """json.loads turns 5.0 into float (rejected above) but also accepts 1e2 as float —
    both are invalid Int32 tokens for .NET, which the type check already covers."""


def parse_record(text: str, fields: dict[str, str]) -> Optional[dict]:
    """Deserialize into a record with the given ``{name: "string"|"int"}`` members.
    Returns None for a JSON ``null`` root; raises NetJsonError like .NET would."""
    val = loads_strict(text)
    if val is None:
        return None
    if not isinstance(val, dict):
        kind = {list: "StartArray", str: "String", int: "Number", float: "Number", bool: "True"}.get(type(val), "Value")
        raise NetJsonError(f"The JSON value could not be converted to the record type. Path: $ | LineNumber: 0 | "
                           f"BytePositionInLine: 1. ({kind})")
    return {k: _typed(val, k, t) for k, t in fields.items()}


RAG_TOOL_CALL = {"action": "string", "namespace": "string", "name": "string", "replicas": "int",
                 "pod": "string", "container": "string"}
AGENT_CALL_ACTION = {"action": "string", "namespace": "string", "pod": "string", "container": "string",
                     "name": "string", "replicas": "int"}
