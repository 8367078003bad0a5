"""Ingestion text processing with the reference's exact semantics.

* :func:`split_by_markdown_headers` — ``Helpers/RagIndex.cs:71-99``: CRLF->LF, new
  section at every line matching ``^\\s*#{1,6}\\s+`` (so YAML front-matter before the
  first header is its own section), sections trimmed, sections longer than 1200
  chars re-split by :func:`chunk_sliding` (800 / 120).  Always returns >= 1 section
  for non-empty input, which makes the caller's sliding-window fallback
  (``RagIndex.cs:39``) dead code — kept for parity (quirk A.7.1).
* :func:`chunk_sliding` — ``RagIndex.cs:101-114``.
* :func:`sanitize` — ``RagIndex.cs:116-122``: strip NULs, trim, redact the three
  prompt-injection phrases (case-insensitive), cap at 2000 chars.

Lengths and slices are in UTF-16 code units like .NET ``string.Length`` /
``Substring`` (identical to Python for BMP text).
"""
from __future__ import annotations

import re

HEADER_RE = re.compile(r"^\s*#{1,6}\s+")
REDACT_RE = re.compile(r"(ignore previous instructions|disregard all prior rules|system prompt)", re.IGNORECASE)

# .NET string.Trim() whitespace: Unicode White_Space (Python's str.strip() default set
# additionally strips \x1c-\x1f; emulate .NET precisely)
_NET_WS = "".join(chr(c) for c in (
    0x09, 0x0A, 0x0B, 0x0C, 0x0D, 0x20, 0x85, 0xA0, 0x1680, 0x2000, 0x2001, 0x2002, 0x2003, 0x2004,
    0x2005, 0x2006, 0x2007, 0x2008, 0x2009, 0x200A, 0x2028, 0x2029, 0x202F, 0x205F, 0x3000))


def net_trim(s: str) -> str:
    return s.strip(_NET_WS)


def u16len(s: str) -> int:
    if s.isascii():
        return len(s)
    return len(s) + sum(1 for ch in s if ord(ch) > 0xFFFF)


def u16slice(s: str, start: int, length: int | None = None) -> str:
    """``s.Substring(start, length)`` in UTF-16 units (surrogate pairs count 2)."""
    if s.isascii() or all(ord(c) <= 0xFFFF for c in s):
        return s[start:] if length is None else s[start:start + length]
    b = s.encode("utf-16-le", "surrogatepass")
    end = len(b) // 2 if length is None else start + length
    return b[2 * start:2 * end].decode("utf-16-le", "surrogatepass")


def chunk_sliding(text: str, size: int, overlap: int) -> list[str]:
    if size <= 0:
        size = 800
    if overlap < 0:
        overlap = 0
    step = max(1, size - overlap)
    n = u16len(text)
    return [u16slice(text, i, min(size, n - i)) for i in range(0, n, step)]


def split_by_markdown_headers(text: str, section_max: int = 1200, resplit_size: int = 800,
                              resplit_overlap: int = 120, newline: str = "\n") -> list[str]:
    """``newline``: what .NET ``StringBuilder.AppendLine`` appends (``Environment.NewLine``:
    "\\n" on Linux — the default here — "\\r\\n" on Windows)."""
    lines = text.replace("\r\n", "\n").split("\n")
    acc: list[str] = []
    sb: list[str] = []
    for line in lines:
        if HEADER_RE.match(line):
            if sb:
                acc.append(net_trim("".join(sb)))
                sb = []
        sb.append(line + newline)
    if sb:
        acc.append(net_trim("".join(sb)))
    out: list[str] = []
    for s in acc:
        if u16len(s) <= section_max:
            out.append(s)
        else:
            out.extend(chunk_sliding(s, resplit_size, resplit_overlap))
    return out


def sanitize(s: str, max_chars: int = 2000) -> str:
    cleaned = net_trim(s.replace("\0", ""))
    cleaned = REDACT_RE.sub("[redacted]", cleaned)
    return u16slice(cleaned, 0, max_chars) if u16len(cleaned) > max_chars else cleaned


def is_blank(s: str) -> bool:
    """``string.IsNullOrWhiteSpace``."""
    return s is None or net_trim(s) == ""


def chunk_document(text: str, chunk_size: int = 800, overlap: int = 120) -> list[str]:
    """Sections of one file, sanitized, blanks dropped (``RagIndex.cs:38-45``)."""
    sections = split_by_markdown_headers(text)
    if not sections:
        sections = chunk_sliding(text, chunk_size, overlap)
    out = []
    for sec in sections:
        clean = sanitize(sec)
        if is_blank(clean):
            continue
        out.append(clean)
    return out
